"""The reference's edge branches, driven through the product's whole-frame loop (bshot_odom) and
checked bit-exact against the oracle, on the host-input path and on the HBM-resident lookahead path:

* fewer valid ratios than K: keypoints = every valid point in ascending-ratio order
  (src/lidar_odometry.cpp:146-153);
* stale normals: a sweep with fewer keypoints than the one before, whose SHOT neighbourhoods read
  surface slots [k, n) of the persistent, mis-indexed normals array that still hold the previous
  sweep's normals (include/bshot_bits.h:59,65-86);
* exact-origin points, skipped by SR (src/lidar_odometry.cpp:63-64) but still surface points;
* isolated points (a lone neighbour = itself: CV ratio 0/0 = NaN, skipped, :121-122);
* exact duplicates of keypoints (the LRF and the SHOT histogram skip d = 0 neighbours);
* an empty sweep and a 4-point sweep (no ISS, LRF < 5 valid neighbours -> NaN SHOT -> 1111 bits,
  RANSAC with < 3 correspondences -> identity, ICP with < 3 points -> no update), followed by
  full sweeps that keep matching against the map (SURVEY.md §5 fault injection)."""
import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

FIELDS = ("n_points", "n_valid_ratios", "n_keypoints", "n_iss", "n_target", "n_mutual", "n_inliers", "icp_iters",
          "gated", "map_size")


def _u(a):
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


def small_frame(seed=7):
    """600 points: 200 isolated points on a 5 m lattice first (index order matters for the stale
    slots), a 380-point cluster, 12 exact duplicates of cluster points and 8 origin points. 392
    valid ratios < K = 600."""
    rng = np.random.default_rng(seed)
    g = np.arange(200)
    iso = np.stack([(g % 20) * 5000.0 - 50000, (g // 20) * 5000.0 + 20000, np.full(200, 500.0)], 1)
    cl = np.array([4000.0, 3000.0, 0.0]) + rng.normal(0, 600, (380, 3))
    cl[:, 2] = np.round(cl[:, 2] / 50) * 50
    return np.concatenate([iso, cl, cl[:12], np.zeros((8, 3))]).astype(np.float32)


def _frames(name):
    A = bshot_py.synth_sweep(0)[0][::4].copy()
    C = bshot_py.synth_sweep(2)[0][::4].copy()
    D = bshot_py.synth_sweep(3)[0][::4].copy()
    B = small_frame()
    if name == "fewer_than_k_stale_normals":
        return [A, B, C, B]
    return [A, np.zeros((0, 3), np.float32), C[:4].copy(), D, B, D]


def _check(f, st, so, od, oo):
    got, exp = [getattr(st, n) for n in FIELDS], [getattr(so, n) for n in FIELDS]
    assert got == exp, (f, dict(zip(FIELDS, zip(got, exp))))
    assert np.array_equal(od.keypoints(), oo.keypoints()), f
    assert np.array_equal(_u(od.ratios()), _u(oo.ratios())), f
    assert np.array_equal(od.bits(), oo.bits()), f
    assert np.array_equal(od.iss(), oo.iss()), f
    tx, tb = od.target()
    ox, ob = oo.target()
    assert np.array_equal(tx, ox) and np.array_equal(tb, ob), f
    q, m = od.inliers()
    oq, om = oo.inliers()
    assert np.array_equal(q, oq) and np.array_equal(m, om), f
    assert _u([st.h_diff, st.t_diff]).tolist() == _u([so.h_diff, so.t_diff]).tolist(), f
    assert np.array_equal(_u(st.T_ransac), _u(so.T_ransac)), f
    assert np.array_equal(_u(st.pose), _u(so.pose)), f


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fewer_than_k_stale_normals", "empty_and_tiny_frames"])
@pytest.mark.parametrize("device", [False, True])
def test_edge_sequence(name, device):
    import torch

    frames = _frames(name)
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=600))
    oo = orc.Odometry(orc.params(num_keypoints=600))
    dev = [torch.from_numpy(x).to("cuda:0") if len(x) else None for x in frames]
    torch.cuda.synchronize()
    ptr = [d.data_ptr() if d is not None else 0 for d in dev]
    try:
        for f, xyz in enumerate(frames):
            if device:
                if f + 1 < len(frames):
                    od.set_next_device(ptr[f + 1], len(frames[f + 1]))
                    if f + 2 < len(frames):
                        od.set_next2_device(ptr[f + 2], len(frames[f + 2]))
                st = od.process_device(ptr[f], len(xyz))
            else:
                st = od.process(xyz)
            so = oo.process(xyz)
            _check(f, st, so, od, oo)
        if name == "fewer_than_k_stale_normals":
            assert 0 < so.n_keypoints < 600 and so.n_valid_ratios == so.n_keypoints
    finally:
        od.close()


def test_stale_normals_matter():
    """Guard for the test above: the small sweep's bits depend on the previous sweep's normals (a
    fresh oracle describing it alone gives different bits), so the stale slots are really read."""
    A, B = _frames("fewer_than_k_stale_normals")[:2]
    o1 = orc.Odometry(orc.params(num_keypoints=600))
    o1.process(A)
    o1.process(B)
    o2 = orc.Odometry(orc.params(num_keypoints=600))
    o2.process(B)
    assert not np.array_equal(o1.bits(), o2.bits())


@pytest.mark.gpu
@pytest.mark.parametrize("host_next", [False, True])
def test_dropped_lookahead_keeps_normals_state(host_next):
    """A lookahead describe whose sweep never comes (wrong next pointer, or the next sweep arrives
    through the host-input path) must leave the persistent normals as the described sweeps left
    them. The dropped prefetch is a full sweep (600 keypoints); the sweep that does come has 392,
    so its SHOT reads slots [392, 600), which must still hold the first sweep's normals."""
    import torch

    A, B, C = _frames("fewer_than_k_stale_normals")[:3]
    dA, dB, dC = (torch.from_numpy(x).to("cuda:0") for x in (A, B, C))
    torch.cuda.synchronize()
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=600))
    oo = orc.Odometry(orc.params(num_keypoints=600))
    try:
        od.set_next_device(dC.data_ptr(), len(C))  # predicted C, but B comes next
        st = od.process_device(dA.data_ptr(), len(A))
        _check(0, st, oo.process(A), od, oo)
        st = od.process(B) if host_next else od.process_device(dB.data_ptr(), len(B))
        _check(1, st, oo.process(B), od, oo)
        st = od.process_device(dC.data_ptr(), len(C))
        _check(2, st, oo.process(C), od, oo)
    finally:
        od.close()
