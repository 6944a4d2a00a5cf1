"""Frame-sharded single sequence (BASELINE config 3 over several GPUs): extraction
contexts each take every W-th sweep (A0-A7 + ISS, with their own lookahead) and ship records; the
chain owner runs A8-A13 on them in sweep order. Every artefact must equal the oracle's sequential
run bit for bit.

The persistent normals array (include/bshot_bits.h:58-87) carries state into a sweep with fewer than
K keypoints: its SHOT reads slots [k, K) as the sweep before it left them. An extracting context
that described another sweep before has other values there, so the owner refuses such a record
(BSHOT_ESTALE, nothing changed) and extracts that sweep itself, from the sequence's own state."""
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


def _check(f, st, so, owner, oo):
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


@pytest.mark.parametrize("W,owner_next", [(1, 0), (2, 0), (3, 0), (2, 1)])
def test_frame_sharded_short_sweeps_match_oracle(W, owner_next):
    """Sweeps with fewer than K keypoints in the middle of the sequence: with one
    extracting context every record is accepted (its stale slots are the sequence's); with W > 1
    the owner refuses the short sweeps' records and extracts them itself, and the whole chain still
    equals the oracle's sequential run bit for bit. owner_next: the caller also gives the owner the
    next sweep (set_next_device), so the owner's context describes a lookahead over its own normals
    array; a refused sweep's own extraction must join and drop it before restoring the sequence's
    state, not adopt it."""
    import torch
    from test_edge_gpu import small_frame

    K = 600
    full = [bshot_py.synth_sweep(f)[0][::4].copy() for f in range(6)]
    B = small_frame()
    xyzs = [full[0], full[1], B, full[2], full[3], B, full[4], B, full[5]]
    F = len(xyzs)
    dev = [torch.from_numpy(x).cuda() for x in xyzs]
    torch.cuda.synchronize()
    prm = bshot_py.default_params(num_keypoints=K)
    ex = [bshot_py.Odometry(0, prm) for _ in range(W)]
    owner = bshot_py.Odometry(0, prm)
    oo = orc.Odometry(orc.params(num_keypoints=K))
    refused = []
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
            if owner_next and f + 1 < F:
                owner.set_next_device(dev[f + 1].data_ptr(), len(xyzs[f + 1]))
            try:
                st = owner.process_record(recs[f])
            except bshot_py.BshotError as e:
                assert e.code == bshot_py.ESTALE, e
                refused.append(f)
                st = owner.process_device(dev[f].data_ptr(), len(xyzs[f]))
            so = oo.process(xyzs[f])
            _check(f, st, so, owner, oo)
            if xyzs[f] is B:
                assert so.n_keypoints < K
    finally:
        for o in ex + [owner]:
            o.close()
    if W == 1:
        assert refused == []
    else:
        assert refused and all(xyzs[f] is B for f in refused), refused


def test_process_record_rejects_garbage():
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    try:
        with pytest.raises(bshot_py.BshotError):
            od.process_record(np.zeros(20, np.float32))
    finally:
        od.close()
