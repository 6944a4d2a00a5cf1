"""Host-side product code (no GPU): top-K selection, RANSAC, keypoint map, bitset layout --
each checked against the oracle or against the reference formula restated here."""
import os

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------------------- top-K (std::sort tail)
@pytest.mark.parametrize("n,k,levels", [(5, 600, 0), (1000, 600, 0), (20000, 600, 7), (129000, 2048, 50),
                                        (129000, 600, 0), (3000, 2048, 3)])
def test_select_topk_matches_std_sort(n, k, levels):
    """bshot_select_topk must reproduce libstdc++ std::sort's (unstable) tail order exactly
    (src/lidar_odometry.cpp:131-153), including the order among equal ratios."""
    rng = np.random.default_rng(n + k + levels)
    r = rng.random(n).astype(np.float32)
    if levels:
        r = (np.floor(r * levels) / levels).astype(np.float32)  # heavy ties
    idx = rng.permutation(n * 2)[:n].astype(np.int32)
    gi, gr = bshot_py.select_topk(idx, r, k)
    ei, er = orc.select_topk(idx, r, k)
    assert np.array_equal(gi, ei) and np.array_equal(gr, er)


def _pattern(kind, n, rng):
    i = np.arange(n)
    x = rng.random(n)
    if kind == "equal":
        return np.ones(n, np.float32)
    if kind == "two":
        return np.where(x < 0.5, 1.0, 0.5).astype(np.float32)
    if kind == "sorted":
        return i.astype(np.float32)
    if kind == "reversed":
        return (n - i).astype(np.float32)
    if kind == "saw":
        return (i % 7).astype(np.float32)
    if kind == "organ":
        return np.minimum(i, n - i).astype(np.float32)
    # CV-like: 1 - min(a, b) / max(a, b) of small counts, many exact 1.0
    a, b = rng.integers(0, 150, n), rng.integers(1, 150, n)
    return (1.0 - np.minimum(a, b) / np.maximum(a, b)).astype(np.float32)


@pytest.mark.parametrize("kind", ["equal", "two", "sorted", "reversed", "saw", "organ", "cv"])
@pytest.mark.parametrize("n,k", [(17, 600), (40, 30), (600, 600), (601, 600), (5000, 2048), (131000, 2048)])
def test_select_topk_patterns_match_std_sort(kind, n, k):
    """The block partition (host/topk.cpp) pairs left and right stoppers as libstdc++'s
    __unguarded_partition does; adversarial value patterns and sizes around k and 16 (the final
    insertion pass's guarded head) against std::sort itself."""
    rng = np.random.default_rng(n * 7 + k)
    r = _pattern(kind, n, rng)
    idx = np.arange(n, dtype=np.int32)
    gi, gr = bshot_py.select_topk(idx, r, k)
    ei, er = orc.select_topk(idx, r, k)
    assert np.array_equal(gi, ei) and np.array_equal(gr.view(np.uint32), er.view(np.uint32))


# ----------------------------------------------------------------------------- RANSAC
def _corr_set(seed, n_src=800, n_corr=400, inlier_frac=0.6, noise=30.0):
    rng = np.random.default_rng(seed)
    src = (rng.random((n_src, 3)) * 60000 - 30000).astype(np.float32)
    a = rng.normal() * 0.05
    R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    t = rng.normal(size=3) * 800
    tgt = (src @ R.T + t + rng.normal(size=src.shape) * noise).astype(np.float32)
    cq = rng.permutation(n_src)[:n_corr].astype(np.int32)
    cm = cq.copy()
    bad = rng.random(n_corr) > inlier_frac
    cm[bad] = rng.integers(0, n_src, bad.sum())
    return src, tgt, cq, cm


@pytest.mark.parametrize("seed,frac", [(1, 0.6), (2, 0.3), (3, 0.9), (4, 0.05)])
def test_ransac_matches_oracle(seed, frac):
    src, tgt, cq, cm = _corr_set(seed, inlier_frac=frac)
    rc, T, iq, im = bshot_py.ransac(src, tgt, cq, cm)
    orc_rc, oT, oq, om = orc.ransac(src, tgt, cq, cm)
    assert rc == orc_rc
    assert np.array_equal(T.view(np.uint32), oT.view(np.uint32))
    assert np.array_equal(iq, oq) and np.array_equal(im, om)


def test_ransac_scores_host_consistent():
    """The host scorer behind bshot_ransac_scores (the GPU kernel's checker): the best-scoring
    hypothesis's count equals the inlier count of the RANSAC result whose model it is."""
    src, tgt, cq, cm = _corr_set(11, inlier_frac=0.6)
    cs, ct = src[cq], tgt[cm]
    hyp = np.arange(3 * 40, dtype=np.int32).reshape(40, 3) % len(cq)
    cnt = bshot_py.ransac_scores(cs, ct, hyp)
    assert cnt.shape == (40,) and cnt.min() >= 0 and cnt.max() <= len(cq)
    # an exact-inlier triple (cm == cq) scores at least its own three correspondences
    good = np.flatnonzero(cq == cm)[:3].astype(np.int32)
    assert bshot_py.ransac_scores(cs, ct, good[None, :])[0] >= 3
    with pytest.raises(bshot_py.BshotError):
        bshot_py.ransac_scores(cs, ct, np.array([[0, 1, len(cq)]], np.int32))


def test_ransac_degenerate():
    src, tgt, cq, cm = _corr_set(5, n_corr=2)
    for ncorr in (0, 1, 2):
        rc, T, iq, _ = bshot_py.ransac(src, tgt, cq[:ncorr], cm[:ncorr])
        orc_rc, oT, oq, _ = orc.ransac(src, tgt, cq[:ncorr], cm[:ncorr])
        assert rc == orc_rc and np.array_equal(T, oT) and len(iq) == len(oq)


# ----------------------------------------------------------------------------- keypoint map
def _block_id_ref(p, prec=10000):
    """src/mymap.cpp:95-105: bitset<64>(int(round(p/prec))*prec), 21 bits per axis."""
    g = [int(np.round(np.float32(x) / np.float32(prec))) * prec for x in p]
    i = ((g[0] & 0xFFFFFFFFFFFFFFFF) << 42) & (0x1FFFFF << 42)
    j = ((g[1] & 0xFFFFFFFFFFFFFFFF) << 21) & (0x1FFFFF << 21)
    k = (g[2] & 0xFFFFFFFFFFFFFFFF) & 0x1FFFFF
    return i | j | k


def test_block_id_packing():
    for p in [(0, 0, 0), (4999, -4999, 1), (5001, 15000, -25001), (-123456, 987654, -1730), (1e6, -1e6, 3e5)]:
        assert bshot_py.KeypointMap.block_id(np.array(p, np.float32)) == _block_id_ref(p), p


def test_map_quantisation_and_suppression():
    m = bshot_py.KeypointMap()
    bits = np.arange(11, dtype=np.uint32) * np.uint32(0x01010101)
    m.add([-15.7, 29.99, 1005.0], 0.5, bits)       # -> (-10, 20, 1000): trunc toward zero, 10 mm grid
    xyz, b = m.query([0, 0, 0])
    assert np.array_equal(xyz, [[-10, 20, 1000]]) and np.array_equal(b[0], bits)
    m.add([300.0, 20.0, 1000.0], 0.4, bits)        # within 800 mm, ratio <= existing -> rejected
    assert m.size() == 1
    m.add([300.0, 20.0, 1000.0], 0.6, bits)        # higher ratio -> kept
    assert m.size() == 2
    m.add([-12.0, 25.0, 1001.0], 0.9, bits ^ 1)    # same quantised position, better ratio -> replaces
    assert m.size() == 2
    m.add([9000.0, 20.0, 1000.0], 0.1, bits)       # > 800 mm away -> kept despite low ratio
    m.add([60000.0, 0, 0], 0.1, bits)               # another block
    assert m.size() == 4
    xyz, _ = m.query([0, 0, 0], 20000.0)           # range query excludes the far block
    assert len(xyz) == 3
    xyz, _ = m.query([60000, 0, 0], 1000.0)
    assert np.array_equal(xyz, [[60000, 0, 0]])


def test_bitset_layout_roundtrip():
    """bit j of bitset<352> <-> word j/32, bit j%32 (bitset<352> stored as 6 x u64 on x86-64)."""
    m = bshot_py.KeypointMap()
    rng = np.random.default_rng(1)
    words = rng.integers(0, 2 ** 32, 11, dtype=np.uint64).astype(np.uint32)
    m.add([0, 0, 0], 0.5, words)
    _, b = m.query([0, 0, 0])
    assert np.array_equal(b[0], words)


def test_map_suppression_random_model():
    """Randomised adds against a direct model of src/mymap.cpp addKeypoint (every keypoint of the
    block within 800 mm and with ratio >= the new one rejects it; same quantised position
    replaces): the cell-bucketed suppression test must keep exactly the same keypoints."""
    rng = np.random.default_rng(7)
    m = bshot_py.KeypointMap()
    blocks = {}
    f32 = np.float32
    for t in range(2500):
        p = rng.uniform(-14000, 14000, 3).astype(np.float32)
        if t % 7 == 0 and t:
            p = prev.copy()  # noqa: F821 -- an earlier position again (replacement path)
        prev = p
        r = float(rng.uniform(0, 1))
        bits = rng.integers(0, 2 ** 32, 11, dtype=np.uint64).astype(np.uint32)
        m.add(p, r, bits)
        q = tuple(f32(int(np.trunc(f32(x) / f32(10))) * 10) for x in p)
        bid = bshot_py.KeypointMap.block_id(np.array(q, np.float32))
        blk = blocks.get(bid)
        if blk is None:
            blocks[bid] = {q: (f32(r), bits)}
            continue
        ok = True
        for k, (rr, _) in blk.items():
            dx, dy, dz = f32(q[0] - k[0]), f32(q[1] - k[1]), f32(q[2] - k[2])
            if np.sqrt(f32(f32(f32(dx * dx) + f32(dy * dy)) + f32(dz * dz))) < f32(800) and f32(r) <= rr:
                ok = False
                break
        if ok:
            blk[q] = (f32(r), bits)
    assert m.size() == sum(len(b) for b in blocks.values())
    xyz, b = m.query([0, 0, 0], 40000.0)
    got = sorted((tuple(x), tuple(w)) for x, w in zip(xyz.tolist(), b.tolist()))
    want = sorted((tuple(float(v) for v in k), tuple(int(v) for v in w)) for blk in blocks.values()
                  for k, (_, w) in blk.items())
    assert got == want


@pytest.mark.parametrize("seed", [1, 2])
def test_map_query_block_scan_order(seed):
    """Map::getKeypoints visiting the map's blocks must return exactly what the reference's
    x/y/z loop of 21^3 block lookups returns (src/mymap.cpp:28-74), in the same order -- including
    blocks whose 21-bit id residues alias positions 2^21 mm away (block-id wraparound)."""
    rng = np.random.default_rng(seed)
    maps = [bshot_py.KeypointMap(), bshot_py.KeypointMap()]
    maps[1].set_query_mode(1)
    span = float(1 << 21)
    for t in range(3000):
        p = rng.uniform(-150000, 150000, 3).astype(np.float32)
        if t % 5 == 0:
            p[rng.integers(0, 3)] += np.float32(span * rng.choice([-1.0, 1.0]))  # aliases a near block id
        bits = rng.integers(0, 2 ** 32, 11, dtype=np.uint64).astype(np.uint32)
        r = float(rng.uniform(0, 1))
        for m in maps:
            m.add(p, r, bits)
    for q in range(40):
        pos = rng.uniform(-120000, 120000, 3).astype(np.float32)
        rng_mm = float(rng.choice([100000.0, 35000.0, 5000.0]))
        a = maps[0].query(pos, rng_mm)
        b = maps[1].query(pos, rng_mm)
        assert len(a[0]) == len(b[0])
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_math_select_forms_match_fdlibm(tmp_path):
    """The SHOT record producers' select forms of atan/atan2/acos (one division for a whole
    wavefront, csrc/bshot_math.h) equal the branchy fdlibm forms bit for bit
    (b-shot-slam_amd/tools/math_sel_check.cpp, 40 M random arguments plus every range boundary)."""
    import subprocess
    exe = tmp_path / "msc"
    src = os.path.join(ROOT, "b-shot-slam_amd", "tools", "math_sel_check.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), src])
    out = subprocess.run([str(exe), "20"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr


def test_umap_order_restatement_matches_libstdcxx(tmp_path):
    """csrc/umap_order.h (the GPU map's per-block iteration order) against this image's libstdc++
    std::unordered_map<Vector3f, ., MapHasher>: bucket counts and iteration order after every insert
    of random 10 mm-grid keys, repeats included (b-shot-slam_amd/tools/umap_order_check.cpp)."""
    import subprocess
    exe = tmp_path / "umcheck"
    src = os.path.join(ROOT, "b-shot-slam_amd", "tools", "umap_order_check.cpp")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", str(exe), src])
    out = subprocess.run([str(exe), "300"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
