"""Known-answer tests that pin the oracle (the CPU restatement in oracle/) with independent
restatements written here from the reference sources, plus numpy/scipy cross-checks.

The reference itself cannot be built in this image (PCL/Eigen/FLANN absent), so the oracle is
"parity unpinned" against PCL; these tests pin every piece of the restatement that can be pinned
independently: FLANN radius-search semantics, the SR ratio formulas, the B-SHOT binarisation
cascade, first-index Hamming argmin + mutual check, the Jacobi eigen-solver and umeyama.
"""
import os
import sys

import numpy as np
import pytest

import oracle_ref as orc


# ----------------------------------------------------------------------------- binarisation
def _bshot_cascade(v):
    """include/bshot_bits.h:144-278, restated: float sums, compared against 0.9*sum in double."""
    f = np.float32
    v0, v1, v2, v3 = (f(x) for x in v)
    s = f(f(f(v0 + v1) + v2) + v3)
    t = 0.9 * float(s)
    if v0 == 0 and v1 == 0 and v2 == 0 and v3 == 0:
        return 0
    rules = [
        (v0, 1), (v1, 2), (v2, 4), (v3, 8),
        (f(v0 + v1), 3), (f(v1 + v2), 6), (f(v2 + v3), 12), (f(v0 + v3), 9), (f(v1 + v3), 10), (f(v0 + v2), 5),
        (f(f(v0 + v1) + v2), 7), (f(f(v1 + v2) + v3), 14), (f(f(v0 + v2) + v3), 13), (f(f(v0 + v1) + v3), 11),
    ]
    for val, b in rules:
        if float(val) > t:
            return b
    return 15


def _bits_ref(shot):
    words = np.zeros(11, np.uint32)
    for j in range(88):
        b = _bshot_cascade(shot[4 * j: 4 * j + 4])
        words[(4 * j) // 32] |= np.uint32(b << ((4 * j) % 32))
    return words


def test_binarize_truth_table():
    # one vector per cascade outcome, in cascade order
    cases = {
        0: [0, 0, 0, 0], 1: [1, 0, 0, 0], 2: [0, 1, 0, 0], 4: [0, 0, 1, 0], 8: [0, 0, 0, 1],
        3: [.5, .5, 0, 0], 6: [0, .5, .5, 0], 12: [0, 0, .5, .5], 9: [.5, 0, 0, .5], 10: [0, .5, 0, .5],
        5: [.5, 0, .5, 0], 7: [.32, .32, .32, .04], 14: [.04, .32, .32, .32], 13: [.32, .04, .32, .32],
        11: [.32, .32, .04, .32], 15: [.25, .25, .25, .25],
    }
    shot = np.zeros((1, 352), np.float32)
    expect = np.zeros(88, np.int64)
    for j, (b, v) in enumerate(cases.items()):
        assert _bshot_cascade(v) == b, (b, v)
        shot[0, 4 * j: 4 * j + 4] = v
        expect[j] = b
    got = orc.binarize(shot)[0]
    nib = np.array([(int(got[(4 * j) // 32]) >> ((4 * j) % 32)) & 15 for j in range(88)])
    assert np.array_equal(nib, expect)
    # NaN group: every comparison false -> 15 (reference falls through to the last branch)
    shot[0, :4] = [np.nan, 0, 0, 0]
    assert (int(orc.binarize(shot)[0][0]) & 15) == 15


def test_binarize_random_vs_restatement():
    rng = np.random.default_rng(7)
    k = 64
    shot = rng.random((k, 352), dtype=np.float32)
    # sparse groups, exact 0.9 boundaries, dominant bins
    shot[rng.random((k, 352)) < 0.5] = 0
    shot[:8, ::4] = 0.9
    shot[:8, 1::4] = 0.1
    shot[8:16, ::4] *= 30
    got = orc.binarize(shot)
    for i in range(k):
        assert np.array_equal(got[i], _bits_ref(shot[i])), i


# ----------------------------------------------------------------------------- radius search
def _bruteforce(xyz, q, r, max_nn):
    d = xyz - q
    d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]  # float32, FLANN L2_3D order
    r2 = np.float32(np.float64(r) * np.float64(r))
    sel = np.nonzero(d2 < r2)[0]
    order = np.lexsort((sel, d2[sel]))
    sel = sel[order]
    if max_nn > 0:
        sel = sel[:max_nn]
    return sel.astype(np.int32), d2[sel]


@pytest.mark.parametrize("max_nn", [0, 30, 300])
def test_radius_search_flann_semantics(max_nn):
    rng = np.random.default_rng(3)
    xyz = (rng.random((6000, 3)) * 4000 - 2000).astype(np.float32)
    xyz[100:200] = xyz[0:100]                  # duplicates -> equal d2 ties broken by index
    xyz[300:400] = np.round(xyz[300:400], -2)  # lattice points -> many equal distances
    queries = np.concatenate([xyz[:40], xyz[300:320], (rng.random((20, 3)) * 5000 - 2500).astype(np.float32)])
    for r in (150.0, 700.0, 3000.0):
        for q in queries:
            gi, gd = orc.radius_search(xyz, q, r, max_nn)
            ei, ed = _bruteforce(xyz, q, r, max_nn)
            assert np.array_equal(gi, ei) and np.array_equal(gd, ed)


def test_radius_search_vs_kdtree():
    cKDTree = pytest.importorskip("scipy.spatial").cKDTree
    rng = np.random.default_rng(11)
    xyz = (rng.random((4000, 3)) * 3000).astype(np.float32)
    tree = cKDTree(xyz.astype(np.float64))
    for q in xyz[:50]:
        gi, _ = orc.radius_search(xyz, q, 400.0, 0)
        ref = set(tree.query_ball_point(q.astype(np.float64), 400.0 - 1e-3))
        # everything well inside the radius is found; nothing beyond it is
        assert ref <= set(gi.tolist())
        assert set(gi.tolist()) <= set(tree.query_ball_point(q.astype(np.float64), 400.0 + 1e-3))


# ----------------------------------------------------------------------------- SR ratios
def _sr_ref(xyz, i, nn, sr_type):
    """src/lidar_odometry.cpp:73-119 restated with float32 scalars in result order."""
    f = np.float32
    sp = xyz[i]
    c = np.zeros(3, np.float32)
    for j in nn:
        c = (c + xyz[j]).astype(np.float32)
    c = (c / f(len(nn))).astype(np.float32)
    t = (sp - c).astype(np.float32)
    if sr_type == 0:
        pos = neg = f(0)
        for j in nn:
            v = (xyz[j] - sp).astype(np.float32)
            dot = f(t[0] * v[0] + f(t[1] * v[1] + t[2] * v[2]))  # Eigen redux: a0 + (a1 + a2)
            if dot > 0:
                pos = f(pos + f(1))
            elif dot < 0:
                neg = f(neg + f(1))
        with np.errstate(invalid="ignore", divide="ignore"):
            return f(f(1) - f(min(pos, neg) / max(pos, neg)))
    ctn = f(np.sqrt(f(t[0] * t[0] + f(t[1] * t[1] + t[2] * t[2]))))
    s = f(0)
    for j in nn:
        v = (xyz[j] - sp).astype(np.float32)
        vn = f(np.sqrt(f(v[0] * v[0] + f(v[1] * v[1] + v[2] * v[2]))))
        if ctn == 0 or vn == 0:
            continue
        dot = f(t[0] * v[0] + f(t[1] * v[1] + t[2] * v[2]))  # Eigen redux: a0 + (a1 + a2)
        s = f(s + (dot if sr_type == 1 else f(dot / f(ctn * vn))))
    return f(abs(s) / f(len(nn)))


@pytest.mark.parametrize("sr_type", [0, 1, 2])
def test_seg_ratio_vs_restatement(sr_type):
    rng = np.random.default_rng(5 + sr_type)
    n = 600
    xyz = (rng.random((n, 3)) * 400).astype(np.float32)
    xyz[:50, 2] = 0  # a plane patch
    xyz[60] = 0      # the origin point is skipped (src/lidar_odometry.cpp:63-64)
    radius, max_nn = 120.0, 30
    idx, rat = orc.seg_ratio(xyz, radius, max_nn, sr_type)
    exp_idx, exp_rat = [], []
    for i in range(n):
        if not xyz[i].any():
            continue
        nn, _ = _bruteforce(xyz, xyz[i], radius, max_nn)
        r = _sr_ref(xyz, i, nn, sr_type)
        if np.isnan(r):
            continue
        exp_idx.append(i)
        exp_rat.append(r)
    assert np.array_equal(idx, np.array(exp_idx, np.int32))
    assert np.array_equal(rat.view(np.uint32), np.array(exp_rat, np.float32).view(np.uint32))


# ----------------------------------------------------------------------------- matching
def test_match_first_index_argmin_and_mutual():
    rng = np.random.default_rng(9)
    a = rng.integers(0, 2 ** 32, (300, 11), dtype=np.uint64).astype(np.uint32)
    b = rng.integers(0, 2 ** 32, (257, 11), dtype=np.uint64).astype(np.uint32)
    b[5] = a[7]
    b[6] = a[7]    # equal-distance duplicates: the first index must win
    a[8] = a[7]
    b[9] = b[11]
    left, right, cq, cm = orc.match(a, b)
    pc = np.vectorize(lambda x: bin(int(x)).count("1"))
    D = pc(a[:, None, :] ^ b[None, :, :]).sum(-1)
    assert np.array_equal(left, D.argmin(1)) and np.array_equal(right, D.argmin(0))
    mutual = [i for i in range(len(a)) if right[left[i]] == i]
    assert np.array_equal(cq, mutual) and np.array_equal(cm, left[mutual])
    assert left[7] == 5 and right[5] == 7


# ----------------------------------------------------------------------------- eigen / umeyama
def test_jacobi_eigen_vs_numpy():
    rng = np.random.default_rng(13)
    for t in range(200):
        m = rng.normal(size=(3, 3)) * (10.0 ** rng.integers(-3, 6))
        a = m @ m.T
        if t % 10 == 0:
            a = np.diag(rng.random(3))
        w, v = orc.eig3(a)
        we = np.linalg.eigvalsh(a)
        assert np.allclose(w, we, rtol=1e-11, atol=1e-12 * abs(we).max())
        assert np.allclose(v.T @ v, np.eye(3), atol=1e-12)
        assert np.allclose(a @ v, v * w, atol=1e-9 * abs(we).max())


def _rot(rng):
    q, _ = np.linalg.qr(rng.normal(size=(3, 3)))
    return q * np.sign(np.linalg.det(q))


@pytest.mark.parametrize("use_float", [False, True])
def test_umeyama_recovers_rigid_transform(use_float):
    rng = np.random.default_rng(17)
    tol = 2e-3 if use_float else 1e-9
    for _ in range(50):
        R, t = _rot(rng), rng.normal(size=3) * 1000
        src = rng.normal(size=(40, 3)) * 5000
        dst = src @ R.T + t
        T = orc.umeyama(src, dst, use_float)
        assert np.allclose(T[:3, :3], R, atol=tol * 1e-3 if use_float else tol)
        assert np.allclose(T[:3, 3], t, atol=tol * 10)
        assert np.array_equal(T[3], [0, 0, 0, 1])
    # noisy: matches the numpy Kabsch/SVD least-squares solution
    src = rng.normal(size=(100, 3)) * 3000
    R, t = _rot(rng), rng.normal(size=3) * 500
    dst = src @ R.T + t + rng.normal(size=(100, 3)) * 20
    sm, dm = src.mean(0), dst.mean(0)
    U, _, Vt = np.linalg.svd((dst - dm).T @ (src - sm))
    S = np.diag([1, 1, np.sign(np.linalg.det(U @ Vt))])
    Re = U @ S @ Vt
    T = orc.umeyama(src, dst, False)
    assert np.allclose(T[:3, :3], Re, atol=1e-10) and np.allclose(T[:3, 3], dm - Re @ sm, atol=1e-7)


@pytest.mark.skipif(bool(os.environ.get("ORACLE_LIB")), reason="already running under the sanitizer build")
def test_oracle_under_sanitizers():
    """the CPU restatement built with AddressSanitizer + UndefinedBehaviorSanitizer
    (oracle/Makefile `sanitize`) runs the oracle's CPU tests -- known-answer tests, host checks, the
    golden fixtures, the preprocessor and capture restatements, the edge frames -- without a report."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "oracle"), "sanitize"])
    pre = ":".join(subprocess.check_output(["gcc", f"-print-file-name={n}"], text=True).strip()
                   for n in ("libasan.so", "libubsan.so"))
    env = dict(os.environ, ORACLE_LIB=os.path.join(root, "oracle", "build", "asan", "liboracle.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               LD_PRELOAD=pre)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider",
                        "-k", "oracle_kat or host or golden or edge or preprocess or velodyne",
                        os.path.join(root, "tests")], env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
