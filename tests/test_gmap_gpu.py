"""§8f row 1: the keypoint map on the GPU (csrc/gmap.hip) against the oracle's Map
(src/mymap.cpp:4-105 restated with libstdc++ containers).

Mode 1 (the default) keeps every block in the iteration order of the reference's
std::unordered_map (csrc/umap_order.h), so the matching targets -- positions, descriptors and their
ORDER, which decides first-index Hamming ties -- equal the host map's bit for bit, and so do the
poses. Mode 2 emits blocks in first-insert order (canonical; checked against the oracle's canonical
mode). Mode 0 is the host map. The 1000-frame config-3 replay (test_sequence_gpu.py) runs mode 1."""
import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

pytestmark = pytest.mark.gpu


def _u(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


@pytest.mark.parametrize("mode", [1, 2, 0])
def test_gpu_map_modes_vs_oracle(mode):
    frames = [bshot_py.synth_sweep(f)[0][::2].copy() for f in range(8)]
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=800))
    od.set_option("gpu_map", mode)
    oo = orc.Odometry(orc.params(num_keypoints=800, map_canonical=1 if mode == 2 else 0))
    try:
        for f, xyz in enumerate(frames):
            st = od.process(xyz)
            so = oo.process(xyz)
            assert (st.n_target, st.n_mutual, st.n_inliers, st.map_size) == (so.n_target, so.n_mutual, so.n_inliers,
                                                                             so.map_size), f
            tx, tb = od.target()
            ox, ob = oo.target()
            assert np.array_equal(_u(tx), _u(ox)) and np.array_equal(tb, ob), f
            assert np.array_equal(_u(st.pose), _u(so.pose)), f
    finally:
        od.close()


def test_gpu_map_lookahead_full_size():
    """Mode 1 in the throughput pipeline (HBM-resident sweeps, depth-2 lookahead), full-size sweeps."""
    import torch

    frames = [bshot_py.synth_sweep(f)[0] for f in range(30, 36)]
    dev = [torch.from_numpy(x).to("cuda:0") for x in frames]
    torch.cuda.synchronize()
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=2048))
    oo = orc.Odometry(orc.params(num_keypoints=2048))
    try:
        for f, (xyz, d) in enumerate(zip(frames, dev)):
            if f + 1 < len(dev):
                od.set_next_device(dev[f + 1].data_ptr(), len(frames[f + 1]))
                if f + 2 < len(dev):
                    od.set_next2_device(dev[f + 2].data_ptr(), len(frames[f + 2]))
            st = od.process_device(d.data_ptr(), len(xyz))
            so = oo.process(xyz)
            assert (st.n_target, st.map_size, st.n_inliers) == (so.n_target, so.map_size, so.n_inliers), f
            tx, tb = od.target()
            ox, ob = oo.target()
            assert np.array_equal(_u(tx), _u(ox)) and np.array_equal(tb, ob), f
            assert np.array_equal(_u(st.pose), _u(so.pose)), f
    finally:
        od.close()
