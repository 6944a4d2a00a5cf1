"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py from the oracle).

CPU: the oracle still reproduces its committed vectors (regression pin of the restatement).
GPU: the product path, called through the C ABI, reproduces the same vectors bit for bit."""
import os

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def stages():
    return _load("stages_8k.npz")


@pytest.fixture(scope="module")
def seq():
    return _load("sequence_3f.npz")


def _u(a):
    return np.ascontiguousarray(a).view(np.uint32)


# ----------------------------------------------------------------------------- oracle (CPU)
def test_oracle_reproduces_stage_fixture(stages):
    g = stages
    k = int(g["k"])
    for tag in ("a", "b"):
        xyz = g[f"xyz_{tag}"]
        sr_idx, sr_ratio = orc.seg_ratio(xyz)
        assert np.array_equal(sr_idx, g[f"sr_idx_{tag}"]) and np.array_equal(_u(sr_ratio), _u(g[f"sr_ratio_{tag}"]))
        kp_idx, _ = orc.select_topk(sr_idx, sr_ratio, k)
        assert np.array_equal(kp_idx, g[f"kp_idx_{tag}"])
        kps = xyz[kp_idx]
        nrm = orc.normals(xyz, kps)
        assert np.array_equal(_u(nrm), _u(g[f"normals_{tag}"]))
        shot, rf = orc.shot(xyz, nrm, kps)
        assert np.array_equal(_u(shot), _u(g[f"shot_{tag}"])) and np.array_equal(_u(rf), _u(g[f"rf_{tag}"]))
        assert np.array_equal(orc.binarize(shot), g[f"bits_{tag}"])
        assert np.array_equal(orc.iss(xyz)[0], g[f"iss_idx_{tag}"])
    left, right, cq, cm = orc.match(g["bits_b"], g["bits_a"])
    for a, b in ((left, "left"), (right, "right"), (cq, "corr_q"), (cm, "corr_m")):
        assert np.array_equal(a, g[b])


def test_oracle_reproduces_sequence_fixture(seq):
    od = orc.Odometry(orc.params(num_keypoints=int(seq["k"])))
    for f in range(3):
        st = od.process(seq[f"xyz_{f}"])
        assert np.array_equal(_u(np.array(st.pose, np.float32)), _u(seq[f"pose_{f}"].reshape(-1)))
        assert np.array_equal(_u(np.array(st.T_ransac, np.float32)), _u(seq[f"T_ransac_{f}"].reshape(-1)))
        assert np.array_equal(od.keypoints(), seq[f"kps_{f}"]) and np.array_equal(od.bits(), seq[f"bits_{f}"])
        q, m = od.inliers()
        assert np.array_equal(q, seq[f"inl_q_{f}"]) and np.array_equal(m, seq[f"inl_m_{f}"])


def corr_stats_restated(kps, tgt, q, m, T):
    """evaluate_corr_ (src/lidar_odometry.cpp:303-330) restated in numpy float32, independently of the
    oracle: pcl::transformPointCloud's ((m00 x + m01 y) + m02 z) + m03 per row, Eigen's
    squaredNorm order a0 + (a1 + a2), float sums in corr order divided by (float)size, median at
    size / 2 of the sorted distances."""
    f32 = np.float32
    T = np.asarray(T, np.float32).reshape(4, 4)
    dv = []
    avg = f32(0)
    for i, j in zip(q, m):
        p = kps[i]
        a = [((T[r, 0] * p[0] + T[r, 1] * p[1]) + T[r, 2] * p[2]) + T[r, 3] for r in range(3)]
        d = [f32(a[r] - tgt[j][r]) for r in range(3)]
        dist = f32(np.sqrt(d[0] * d[0] + (d[1] * d[1] + d[2] * d[2])))
        dv.append(dist)
        avg = f32(avg + dist)
    n = len(dv)
    if n == 0:
        return 0, np.nan, np.nan, np.nan
    avg = f32(avg / f32(n))
    sd = f32(0)
    for dist in dv:
        sd = f32(sd + (dist - avg) * (dist - avg))
    sd = f32(np.sqrt(f32(sd / f32(n))))
    return n, avg, sd, sorted(dv)[n // 2]


@pytest.mark.parametrize("eval_icp", [1, 0])
def test_oracle_corr_stats_match_restatement(seq, eval_icp):
    """The oracle's evaluate_corr_ statistics against the numpy restatement above, on the 3-frame
    sequence fixture (T_best_ with eval_icp, the RANSAC transform without)."""
    od = orc.Odometry(orc.params(num_keypoints=int(seq["k"]), eval_icp=eval_icp))
    for f in range(3):
        st = od.process(seq[f"xyz_{f}"])
        q, m = od.inliers()
        tgt, _ = od.target()
        T = np.array(st.pose if eval_icp else st.T_ransac, np.float32)
        n, avg, sd, med = corr_stats_restated(od.keypoints(), tgt, q, m, T)
        assert st.corr_n == n == len(q), f
        got = np.array([st.corr_avg, st.corr_sd, st.corr_med], np.float32)
        assert np.array_equal(_u(got), _u(np.array([avg, sd, med], np.float32))), (f, got, avg, sd, med)


# ----------------------------------------------------------------------------- product (GPU)
@pytest.mark.gpu
def test_gpu_reproduces_stage_fixture(stages):
    g = stages
    k = int(g["k"])
    bits = {}
    for tag in ("a", "b"):
        ctx = bshot_py.Context(0)  # fresh context: the persistent normals array starts zeroed
        xyz = g[f"xyz_{tag}"]
        ctx.set_cloud(xyz)
        sr_idx, sr_ratio = ctx.seg_ratio()
        assert np.array_equal(sr_idx, g[f"sr_idx_{tag}"]) and np.array_equal(_u(sr_ratio), _u(g[f"sr_ratio_{tag}"]))
        kp_idx, _ = bshot_py.select_topk(sr_idx, sr_ratio, k)
        assert np.array_equal(kp_idx, g[f"kp_idx_{tag}"])
        b, shot, rf = ctx.describe(xyz[kp_idx])
        assert np.array_equal(_u(ctx.normals(len(xyz))), _u(g[f"normals_{tag}"]))
        assert np.array_equal(_u(rf), _u(g[f"rf_{tag}"]))
        assert np.array_equal(_u(shot), _u(g[f"shot_{tag}"]))
        assert np.array_equal(b, g[f"bits_{tag}"])
        assert np.array_equal(ctx.iss(), g[f"iss_idx_{tag}"])
        bits[tag] = b
        left, right, cq, cm = ctx.match(g["bits_b"], g["bits_a"])
        for a, nm in ((left, "left"), (right, "right"), (cq, "corr_q"), (cm, "corr_m")):
            assert np.array_equal(a, g[nm])
        ctx.close()


@pytest.mark.gpu
def test_gpu_reproduces_sequence_fixture(seq):
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=int(seq["k"])))
    for f in range(3):
        st = od.process(seq[f"xyz_{f}"])
        assert np.array_equal(od.keypoints(), seq[f"kps_{f}"]), f
        assert np.array_equal(od.bits(), seq[f"bits_{f}"]), f
        q, m = od.inliers()
        assert np.array_equal(q, seq[f"inl_q_{f}"]) and np.array_equal(m, seq[f"inl_m_{f}"]), f
        assert np.array_equal(_u(np.array(st.T_ransac, np.float32)), _u(seq[f"T_ransac_{f}"].reshape(-1))), f
        assert np.array_equal(_u(np.array(st.pose, np.float32)), _u(seq[f"pose_{f}"].reshape(-1))), f
    od.close()


def test_sequence_1000f_covers_gate_branches():
    """The config-3 golden (tests/golden/sequence_1000f.npz, replayed bit-exact on the GPU by
    tests/test_sequence_gpu.py) drives every branch of the gate (src/lidar_odometry.cpp:273-289):
    NaN h_diff (acos of a rounded T_ij(1,1) > 1: every comparison false, so not gated by the
    angle test), gated frames (previous pose kept, map not flagged) and accepted frames."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sequence_1000f.npz"))
    fields = [str(x) for x in g["stat_fields"]]
    gated = g["stats"][:, fields.index("gated")]
    nan_h = np.isnan(g["h_diff"])
    assert nan_h.sum() >= 1
    assert (gated == 1).sum() >= 1 and (gated == 0).sum() >= 1
    # a NaN-h_diff frame is gated only by t_diff > 1200 or < 15 correspondences
    t = g["t_diff"]
    inl = g["stats"][:, fields.index("n_inliers")]  # corr_ = the RANSAC inliers
    for f in np.flatnonzero(nan_h):
        assert gated[f] == (1 if (t[f] > 1200 or inl[f] < 15) else 0), f
