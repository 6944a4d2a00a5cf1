"""Frame-sharded single sequence (BASELINE config 3 over several GPUs): extraction
contexts each take every W-th sweep (A0-A7 + ISS, with their own lookahead) and ship records; the
chain owner runs A8-A13 on them in sweep order. Every artefact must equal the oracle's sequential
run bit for bit (the sweeps carry K keypoints each, so the persistent normals array carries no
state across sweeps, bshot_abi.h)."""
import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

pytestmark = pytest.mark.gpu


def _u(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("W", [2, 3])
def test_frame_sharded_sequence_matches_oracle(W):
    import torch
    K, F = 600, 7
    xyzs = [bshot_py.synth_sweep(f)[0] for f in range(F)]
    dev = [torch.from_numpy(x).cuda() for x in xyzs]
    torch.cuda.synchronize()
    prm = bshot_py.default_params(num_keypoints=K)
    ex = [bshot_py.Odometry(0, prm) for _ in range(W)]
    owner = bshot_py.Odometry(0, prm)
    oo = orc.Odometry(orc.params(num_keypoints=K))
    try:
        recs = {}
        for r in range(W):
            mine = list(range(r, F, W))
            for i, f in enumerate(mine):
                if i + 1 < len(mine):
                    ex[r].set_next_device(dev[mine[i + 1]].data_ptr(), len(xyzs[mine[i + 1]]))
                recs[f] = ex[r].extract_device(dev[f].data_ptr(), len(xyzs[f]))
            ex[r].drain()
        for f in range(F):
            st = owner.process_record(recs[f])
            so = oo.process(xyzs[f])
            assert st.n_keypoints == K, f
            for name in ("n_points", "n_valid_ratios", "n_keypoints", "n_iss", "n_target", "n_mutual", "n_inliers",
                         "icp_iters", "gated", "map_size"):
                assert getattr(st, name) == getattr(so, name), (f, name, getattr(st, name), getattr(so, name))
            assert np.array_equal(owner.keypoints(), oo.keypoints()), f
            assert np.array_equal(_u(owner.ratios()), _u(oo.ratios())), f
            assert np.array_equal(owner.bits(), oo.bits()), f
            assert np.array_equal(owner.iss(), oo.iss()), f
            tx, tb = owner.target()
            ox, ob = oo.target()
            assert np.array_equal(tx, ox) and np.array_equal(tb, ob), f
            q, m = owner.inliers()
            oq, om = oo.inliers()
            assert np.array_equal(q, oq) and np.array_equal(m, om), f
            assert np.array_equal(_u(np.array(st.pose)), _u(np.array(so.pose))), f
    finally:
        for o in ex + [owner]:
            o.close()


def test_process_record_rejects_garbage():
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    try:
        with pytest.raises(bshot_py.BshotError):
            od.process_record(np.zeros(20, np.float32))
    finally:
        od.close()
