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


@pytest.mark.parametrize("mode,slots0", [(1, None), (2, None), (0, None), (1, 64)])
def test_gpu_map_modes_vs_oracle(mode, slots0):
    """slots0: the map's up-front slot reservation (option gmap_slots0, default 2^20); 64 makes the
    map grow by doubling, its contents kept, over the sequence's inserts."""
    frames = [bshot_py.synth_sweep(f)[0][::2].copy() for f in range(8)]
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=800))
    od.set_option("gpu_map", mode)
    if slots0 is not None:
        od.set_option("gmap_slots0", slots0)
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


def _rec(xyz, ratio, rng):
    """map-delta records (x, y, z on the 10 mm grid, ratio, 11 descriptor words) as float32 rows"""
    n = len(xyz)
    rec = np.zeros((n, 15), np.float32)
    rec[:, :3] = xyz
    rec[:, 3] = ratio
    rec[:, 4:] = rng.integers(0, 2 ** 32, (n, 11), dtype=np.uint64).astype(np.uint32).view(np.float32)
    return rec


def _host_add(hm, rec):
    for r in rec:
        hm.add(r[:3].copy(), float(r[3]), r[4:].view(np.uint32).copy())


def test_gmap_crafted_inserts_vs_host_map():
    """k_gmap_insert's subtle paths against the host Map (myslam::Map restated, itself checked against
    libstdc++'s unordered_map in test_host.py), through GPU replica inserts of crafted batches:
    exact-position repeats with rising ratios (operator[] replacement), several candidates of one
    batch in one 800 mm neighbourhood (suppression in sweep order), and a block growing past 2400
    members in one batch (rehashes up to 5087 buckets inside the workgroup's LDS image)."""
    rng = np.random.default_rng(3)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    hm = bshot_py.KeypointMap()
    try:
        batches = []
        # exact repeats and rising ratios, plus near neighbours in the same batch
        base = np.array([[120.0, 340.0, -50.0], [900.0, 340.0, -50.0], [120.0, 1500.0, 10.0]], np.float32)
        pts = np.concatenate([base, base, base + [10.0, 0.0, 0.0], base]).astype(np.float32)
        batches.append(_rec(pts, np.linspace(0.1, 0.9, len(pts)).astype(np.float32), rng))
        batches.append(_rec(base, np.array([0.95, 0.05, 0.5], np.float32), rng))
        # one block (ids round(p / 1e4)) past 2400 members: rising ratios admit every candidate
        g = np.stack(np.meshgrid(np.arange(-4800, 4800, 360), np.arange(-4800, 4800, 360), np.arange(-1000, 1000, 500)),
                     -1).reshape(-1, 3).astype(np.float32) + [20000.0, 0.0, 0.0]
        g = g[rng.permutation(len(g))][:2600]
        batches.append(_rec(g, np.linspace(0.01, 0.99, len(g)).astype(np.float32), rng))
        # a later batch into the same dense block: exact repeats of members and new points
        again = np.concatenate([g[:50], g[100:150] + [10.0, 10.0, 0.0]]).astype(np.float32)
        batches.append(_rec(again, rng.uniform(0, 1, len(again)).astype(np.float32), rng))
        for rec in batches:
            od.gpu_replica_insert(0, rec)
            _host_add(hm, rec)
            assert od.gpu_replica_size(0) == hm.size()
            for pos in ([0.0, 0.0, 0.0], [20000.0, 0.0, 0.0]):
                gx, gb = od.gpu_replica_query(0, np.array(pos, np.float32))
                hx, hb = hm.query(np.array(pos, np.float32))
                assert np.array_equal(_u(gx), _u(hx)) and np.array_equal(gb, hb)
        assert hm.size() > 2400
    finally:
        od.close()


def test_gmap_block_crossing_small_image_limit():
    """a block whose members plus the batch fit the small LDS image before the insert
    (<= 1024) belongs to the small-image launch alone, even when the insert takes it past 1024; a
    block already past 1024 goes to the full-image launch. Both against the host Map."""
    rng = np.random.default_rng(11)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    hm = bshot_py.KeypointMap()
    try:
        g = np.stack(np.meshgrid(np.arange(-4800, 4800, 300), np.arange(-4800, 4800, 300), np.arange(-900, 900, 600)),
                     -1).reshape(-1, 3).astype(np.float32) + [-30000.0, 10000.0, 0.0]
        g = g[rng.permutation(len(g))]
        assert len(g) >= 1300
        r = np.linspace(0.01, 0.99, 1300).astype(np.float32)  # rising: every candidate is admitted
        parts = [(g[:600], r[:600]), (g[600:1000], r[600:1000]),  # 600 + 400 <= 1024 before the insert
                 (g[1000:1100], r[1000:1100]),                     # 1000 + 100 > 1024: the full image
                 (np.concatenate([g[:40], g[1100:1300]]), np.concatenate([r[:40] + 0.5, r[1100:1300]]))]
        for pts, rat in parts:
            rec = _rec(pts, rat, rng)
            od.gpu_replica_insert(0, rec)
            _host_add(hm, rec)
            assert od.gpu_replica_size(0) == hm.size()
            for pos in ([-30000.0, 10000.0, 0.0], [-25000.0, 5000.0, 0.0]):
                gx, gb = od.gpu_replica_query(0, np.array(pos, np.float32))
                hx, hb = hm.query(np.array(pos, np.float32))
                assert np.array_equal(_u(gx), _u(hx)) and np.array_equal(gb, hb)
        assert hm.size() > 1100
    finally:
        od.close()


def test_gmap_large_batches_both_sort_paths():
    """A batch's block ids are ordered by a one-workgroup LDS sort up to 4096 keypoints and by the
    rocprim radix sort past that; both must leave the replica equal to the host Map (sizes, and the
    reference's block loop around several positions)."""
    rng = np.random.default_rng(5)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    hm = bshot_py.KeypointMap()
    try:
        for k in (4096, 6000, 1):
            pts = np.round(rng.uniform(-6000, 6000, (k, 3))) * 10.0  # on the map's 10 mm grid
            pts[:, 2] = np.round(rng.uniform(-300, 300, k)) * 10.0
            pts = (pts + 0.0).astype(np.float32)  # +0, as the 10 mm quantisation writes it (never -0)
            rec = _rec(pts, rng.uniform(0, 1, k).astype(np.float32), rng)
            od.gpu_replica_insert(0, rec)
            _host_add(hm, rec)
            assert od.gpu_replica_size(0) == hm.size()
            for pos in ([0.0, 0.0, 0.0], [40000.0, -30000.0, 0.0], [-55000.0, 52000.0, 1000.0]):
                gx, gb = od.gpu_replica_query(0, np.array(pos, np.float32))
                hx, hb = hm.query(np.array(pos, np.float32))
                assert np.array_equal(_u(gx), _u(hx)) and np.array_equal(gb, hb)
    finally:
        od.close()


def test_gmap_block_capacity_error_surfaces():
    """A 10 m block holds at most 4096 members in the GPU map (the insert workgroup's LDS image;
    DESIGN.md §3). Going past it is reported (BSHOT_ECAP), never silently dropped."""
    rng = np.random.default_rng(4)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=64))
    try:
        g = np.stack(np.meshgrid(np.arange(-4900, 4900, 240), np.arange(-4900, 4900, 240), np.arange(-1000, 1000, 500)),
                     -1).reshape(-1, 3).astype(np.float32)
        assert len(g) > 4096
        with pytest.raises(bshot_py.BshotError):
            od.gpu_replica_insert(0, _rec(g, np.linspace(0.01, 0.99, len(g)).astype(np.float32), rng))
    finally:
        od.close()
