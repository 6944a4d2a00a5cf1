"""GPU parity of each hot-path stage against the CPU restatement (oracle/), same inputs.

Tiers (SURVEY.md §8c / DESIGN.md): integer and index work bit-exact; the float stages are ALSO
expected bit-exact because device and oracle share one documented operation order
(-ffp-contract=off, IEEE +-*/ sqrt, identical transcendental algorithms); the stated tolerance
below (SHOT |d| <= 1e-5, normals <= 1e-5) is the contract floor, bit-equality is asserted where
the convention guarantees it."""
import os

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = bshot_py.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def cloud():
    pc, _ = bshot_py.synth_sweep(3)
    return pc


@pytest.fixture(scope="module")
def sr_ref(cloud):
    return orc.seg_ratio(cloud)


@pytest.mark.parametrize("ladder", [4, 2])
def test_seg_ratio_bit_exact(ctx, cloud, sr_ref, ladder):
    ctx.set_option("ladder_grids", ladder)  # 4 nested grids / 7 radii (default) and 2 grids / 4 radii
    ctx.set_cloud(cloud)
    idx, rat = ctx.seg_ratio()
    ridx, rrat = sr_ref
    assert len(idx) == len(ridx)
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(rat.view(np.uint32), rrat.view(np.uint32))
    ctx.set_option("ladder_grids", 4)


@pytest.mark.parametrize("opts", [{"sr_xcd_chunk": 0}, {"sr_xcd_chunk": 4096}, {"sr_start": 0}, {"sr_start": 300},
                                  {"sr_blocks": 1024}, {"sr_run": 1}, {"sr_run": 3}, {"sr_run": 64},
                                  {"sr_run": 64, "sr_bratio": 101}, {"sr_bratio": 283}, {"sr_bratio": 1000},
                                  {"sr_run": 16, "sr_blocks": 512, "sr_xcd_chunk": 0}])
def test_seg_ratio_schedules_agree(ctx, cloud, sr_ref, opts):
    """The SR launch's query schedule (XCD-local chunks or round-robin, a persistent grid), the
    ladder's start step, and the runs of cell-order queries whose radii chain from their
    predecessor's max_nn-th distance (sr_run, with the bounded pass's grid choice sr_bratio) only
    change the work done, never a ratio."""
    defaults = {"sr_xcd_chunk": 1024, "sr_start": 80, "sr_blocks": 0, "sr_run": 4, "sr_bratio": 200}
    try:
        for k, v in opts.items():
            ctx.set_option(k, v)
        ctx.set_cloud(cloud)
        idx, rat = ctx.seg_ratio()
    finally:
        for k in opts:
            ctx.set_option(k, defaults[k])
    ridx, rrat = sr_ref
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(rat.view(np.uint32), rrat.view(np.uint32))


def _edge_cloud():
    """Sparse far points, a dense clump whose neighbourhoods overflow the kNN list (> KNN_CAP keys:
    the streaming selection), exact duplicates, origin points, NaN/inf rows and points beyond the
    ladder keys' range (no grid cell: ratio NaN)."""
    rng = np.random.default_rng(11)
    far = rng.uniform(-90000, 90000, (3000, 3))
    clump = np.array([2000.0, -1000.0, 300.0]) + rng.normal(0, 250, (6000, 3))
    plane = np.stack([rng.uniform(-8000, 8000, 20000), rng.uniform(-8000, 8000, 20000), np.full(20000, -1800.0)], 1)
    dup = clump[:40]
    bad = np.array([[np.nan, 0, 0], [0, np.inf, 0], [0, 0, -np.inf], [6e7, 0, 0], [0, -6e7, 100]])
    xyz = np.concatenate([far, clump, plane, dup, np.zeros((5, 3)), bad]).astype(np.float32)
    return xyz[rng.permutation(len(xyz))]


@pytest.mark.parametrize("sr_type,run", [(0, 8), (1, 8), (2, 8), (0, 1), (0, 256)])
def test_seg_ratio_edge_cases(sr_type, run):
    xyz = _edge_cloud()
    ridx, rrat = orc.seg_ratio(xyz, sr_type=sr_type)
    c = bshot_py.Context(0, bshot_py.default_params(sr_type=sr_type))
    try:
        c.set_option("sr_run", run)
        c.set_cloud(xyz)
        idx, rat = c.seg_ratio()
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(rat.view(np.uint32), rrat.view(np.uint32))
    finally:
        c.close()


def test_seg_ratio_point_beyond_grid_range_fails_loudly():
    """A finite point beyond the grids' coordinate range (2^20 finest cells, +-98 km at the default
    radius) is in no cell: the sweep fails with BSHOT_ECAP rather than computing ratios without it."""
    rng = np.random.default_rng(5)
    xyz = rng.normal(0, 2000, (5000, 3)).astype(np.float32)
    c = bshot_py.Context(0)
    try:
        c.set_cloud(xyz)
        c.seg_ratio()  # in range: fine
        xyz[17] = (2.0e8, 0.0, 0.0)
        c.set_cloud(xyz)
        with pytest.raises(bshot_py.BshotError, match="coordinate range"):
            c.seg_ratio()
    finally:
        c.close()


def test_topk_keypoints_exact(sr_ref):
    ridx, rrat = sr_ref
    for k in (600, 2048):
        a = bshot_py.select_topk(ridx, rrat, k)
        b = orc.select_topk(ridx, rrat, k)
        np.testing.assert_array_equal(a[0], b[0])


@pytest.mark.parametrize("iss_grid,xcd", [(1, 1024), (0, 1024), (1, 0), (1, 64)])
def test_iss_exact(ctx, cloud, iss_grid, xcd):
    """ISS on the SR ladder's finest grid (default) and on a grid of its own; the lane kernel's
    points in XCD-local chunks of cell order (1024 default, 64) or in plain block order (0)."""
    ctx.set_option("iss_grid", iss_grid)
    ctx.set_option("iss_xcd_chunk", xcd)
    try:
        ctx.set_cloud(cloud)
        got = ctx.iss()
    finally:
        ctx.set_option("iss_grid", 1)
        ctx.set_option("iss_xcd_chunk", 1024)
    ref, _ = orc.iss(cloud)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("k,nseg", [(600, 1), (2048, 1), (2048, 0)])  # k ascending: the module context's persistent normals array must not hold stale slots from a larger K
def test_describe_parity(ctx, cloud, sr_ref, k, nseg):
    """Load-balanced SHOT: bucketed gather + in-bucket rank, chunked LRF, records + ordered apply
    (7 waves compute the records and one applies them, in one workgroup per keypoint: k_hist_fused).
    Normals from the sorted SHOT segments (nseg 1, the default with normal_radius == shot_radius) or
    from their own radius search (k_normals)."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, k)
    kps = cloud[kidx]
    ctx.set_cloud(cloud)
    ctx.set_option("normals_seg", nseg)
    try:
        bits, shot, rf = ctx.describe(kps)
    finally:
        ctx.set_option("normals_seg", 1)
    nrm = ctx.normals(len(cloud))
    rn = orc.normals(cloud, kps)
    # normals: bit-exact by convention (contract tolerance 1e-5)
    assert np.nanmax(np.abs(nrm[:k] - rn[:k])) <= 1e-5
    np.testing.assert_array_equal(np.isnan(nrm), np.isnan(rn))
    same_n = np.all((nrm.view(np.uint32) == rn.view(np.uint32)) | (np.isnan(nrm) & np.isnan(rn)))
    rs, rrf = orc.shot(cloud, rn, kps)
    rb = orc.binarize(rs)
    np.testing.assert_array_equal(np.isnan(rf), np.isnan(rrf))
    assert np.nanmax(np.abs(rf - rrf)) <= 1e-5
    assert np.nanmax(np.abs(shot - rs)) <= 1e-5
    assert same_n, "normals differ in the last bits"
    np.testing.assert_array_equal(rf.view(np.uint32)[~np.isnan(rf)], rrf.view(np.uint32)[~np.isnan(rrf)])
    np.testing.assert_array_equal(shot.view(np.uint32)[~np.isnan(shot)], rs.view(np.uint32)[~np.isnan(rs)])
    np.testing.assert_array_equal(bits, rb)


def test_normals_from_segments_edge_keypoints(ctx, cloud):
    """k_normals_seg on keypoints that are not cloud points: off-surface, isolated (< 3 or no
    neighbours within the radius), duplicated and non-finite. Equal to k_normals and the oracle."""
    rng = np.random.default_rng(21)
    kps = np.concatenate([cloud[rng.choice(len(cloud), 200, replace=False)] + rng.normal(0, 400, (200, 3)),
                          np.array([[9.0e5, 9.0e5, 0.0], [0.0, 0.0, 0.0], [np.nan, 1.0, 2.0], [1.0, np.inf, 2.0]]),
                          cloud[:3], cloud[:3]]).astype(np.float32)
    ctx.set_cloud(cloud)
    out = {}
    for nseg in (1, 0):
        ctx.set_option("normals_seg", nseg)
        bits, shot, rf = ctx.describe(kps)
        out[nseg] = (ctx.normals(len(kps)), bits, shot)
    ctx.set_option("normals_seg", 1)
    rn = orc.normals(cloud, kps)
    for nseg in (1, 0):
        nrm = out[nseg][0]
        np.testing.assert_array_equal(np.isnan(nrm), np.isnan(rn[:len(kps)]))
        ok = ~np.isnan(rn[:len(kps)])
        np.testing.assert_array_equal(nrm.view(np.uint32)[ok], rn[:len(kps)].view(np.uint32)[ok])
    np.testing.assert_array_equal(out[1][1], out[0][1])
    np.testing.assert_array_equal(out[1][2].view(np.uint32), out[0][2].view(np.uint32))


@pytest.mark.parametrize("hint", [1 << 26, 1])
def test_describe_device_plan(ctx, cloud, sr_ref, hint):
    """Describe planned on the device (capacity hint ample) and the re-plan after a device plan
    overflows its capacity (hint 1): both give the host-planned bits (hint 0: no size seen yet, the
    plan is made on the host, as for a context's first describe)."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 2048)
    kps = cloud[kidx]
    ctx.set_cloud(cloud)
    ctx.set_option("dev_plan_hint", 0)
    ref_bits, ref_shot, _ = ctx.describe(kps)
    ctx.set_option("dev_plan_hint", hint)
    bits, shot, _ = ctx.describe(kps)
    np.testing.assert_array_equal(bits, ref_bits)
    np.testing.assert_array_equal(shot.view(np.uint32), ref_shot.view(np.uint32))


def test_match_exact_random_and_ties(ctx):
    """A9 (one-pass k_ham_pair: row and column minima from one distance tile) vs the oracle: sizes
    across the row tiles (512 rows per workgroup), the reference splits and the LDS tiles (128),
    duplicated rows on both sides (first index must win in both directions), all-equal distances."""
    rng = np.random.default_rng(7)
    for na, nb in ((1, 1), (5, 300), (600, 1800), (2048, 4096), (257, 1), (513, 129), (2047, 15001), (4100, 37),
                   (1, 20000), (3000, 3000)):
        a = rng.integers(0, 2**32, (na, 11), dtype=np.uint64).astype(np.uint32)
        b = rng.integers(0, 2**32, (nb, 11), dtype=np.uint64).astype(np.uint32)
        # sparse descriptors (like the degenerate B-SHOT bits) -> many distance ties
        a &= rng.integers(0, 2**32, (na, 11), dtype=np.uint64).astype(np.uint32) & 0x11111111
        b &= rng.integers(0, 2**32, (nb, 11), dtype=np.uint64).astype(np.uint32) & 0x11111111
        b[nb // 2:] = b[: nb - nb // 2]  # duplicated rows: first index must win
        a[na // 2:] = a[: na - na // 2]
        got = ctx.match(a, b)
        ref = orc.match(a, b)
        for g, r in zip(got, ref):
            np.testing.assert_array_equal(g, r)
    a = np.zeros((700, 11), np.uint32)  # every distance 0: left = 0, right = 0, only row 0 mutual
    b = np.zeros((900, 11), np.uint32)
    for g, r in zip(ctx.match(a, b), orc.match(a, b)):
        np.testing.assert_array_equal(g, r)


@pytest.mark.parametrize("device_loop,relay", [(0, 1), (0, 0), (1, 1)])
def test_icp_exact(ctx, cloud, sr_ref, device_loop, relay):
    """A11: ICP (iteration 0 builds candidate lists, later iterations search them) vs the oracle,
    bit for bit: the host's float Umeyama loop (default; its releases read by one workgroup and
    relayed in device memory, or read from host memory by every workgroup: option icp_relay) and the
    device loop (option icp_device)."""
    ctx.set_option("icp_relay", relay)
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 600)
    tgt = cloud[kidx]
    c, s = np.cos(0.01), np.sin(0.01)
    src = (tgt @ np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float32).T + np.array([300, -200, 50], np.float32))
    src = src.astype(np.float32)
    ctx.set_option("icp_device", device_loop)
    try:
        T, it = ctx.icp(src, tgt)
    finally:
        ctx.set_option("icp_device", 0)
        ctx.set_option("icp_relay", 1)
    Tr, itr = orc.icp(src, tgt)
    assert it == itr
    np.testing.assert_array_equal(T.view(np.uint32), Tr.view(np.uint32))


@pytest.mark.parametrize("relay", [1, 0])
def test_icp_host_stall_restarts(ctx, cloud, sr_ref, relay):
    """a host stall longer than the persistent kernel's 1 s wait (the host sleeps 1.3 s
    before releasing iteration 3) makes the kernel exit; the host restarts the iterations from its
    current positions and the result is still the oracle's, bit for bit."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 600)
    tgt = cloud[kidx]
    c, s = np.cos(0.02), np.sin(0.02)
    src = (tgt @ np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float32).T + np.array([600, -300, 80], np.float32))
    src = src.astype(np.float32)
    w0 = ctx.work()
    ctx.set_option("icp_host_delay_ms", 1300)
    ctx.set_option("icp_relay", relay)
    try:
        T, it = ctx.icp(src, tgt)
    finally:
        ctx.set_option("icp_host_delay_ms", 0)
        ctx.set_option("icp_relay", 1)
    w1 = ctx.work()
    Tr, itr = orc.icp(src, tgt)
    assert it == itr and it > 3
    np.testing.assert_array_equal(T.view(np.uint32), Tr.view(np.uint32))
    assert w1[3] - w0[3] >= 1  # the restart happened


def test_icp_iteration_counts_and_sizes(ctx, cloud, sr_ref):
    """A11 device loop (k_icp_loop) vs the oracle's host loop: PCL's iteration cap at 0, 1, 2 and
    beyond the old hand-over's 64 (200: the loop stops on its own convergence test), source counts
    not a multiple of 4 (LDS row tails) and just past the LDS staging (2049: the HBM-chunked
    Umeyama)."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 2100)
    tgt = cloud[kidx]
    c, s = np.cos(0.02), np.sin(0.02)
    rot = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float32)
    for dev in (0, 1):
        ctx.set_option("icp_device", dev)
        try:
            for ns, it_cap in ((2100, 0), (2100, 1), (2100, 2), (2100, 200), (1001, 10), (2049, 10), (2048, 10), (3, 10)):
                src = (tgt[:ns] @ rot.T + np.array([700, -400, 90], np.float32)).astype(np.float32)
                T, it = ctx.icp(src, tgt, max_iter=it_cap)
                Tr, itr = orc.icp(src, tgt, max_iter=it_cap)
                assert it == itr, (dev, ns, it_cap)
                np.testing.assert_array_equal(T.view(np.uint32), Tr.view(np.uint32))
        finally:
            ctx.set_option("icp_device", 0)


@pytest.mark.parametrize("big", [False, True])
def test_icp_grid_edge_cases(big):
    """A11 1-NN on the target grids vs the oracle's brute force: sources far beyond every ball
    (the brute-force scan), exact-duplicate targets (index tie), targets exactly on a ball radius
    (d2 == rs^2 is outside the ball), a non-finite source, sparse and dense targets; sources that
    move beyond their iteration-0 candidate lists fall back to the grid search. big: > 5000 sources
    in dense clusters (candidate lists over capacity)."""
    rng = np.random.default_rng(11)
    tgt = (rng.random((5000, 3)) * [80000, 80000, 4000] - [40000, 40000, 2000]).astype(np.float32)
    tgt[100:110] = tgt[90]  # duplicates
    tgt[200] = [0, 0, 0]
    tgt[201] = [1000, 0, 0]
    src = np.concatenate([tgt[:1500] + rng.normal(0, 300, (1500, 3)), tgt[1500:1600] + 7000.0,
                          [[0, 0, 0], [1000, 0, 0], [500, 0, 0], [2e6, 2e6, 0], [-9e5, 0, 3e5]],
                          tgt[90:91] + 1.0]).astype(np.float32)
    if big:
        src = np.concatenate([src, tgt[:3600] + rng.normal(0, 500, (3600, 3))]).astype(np.float32)
        assert len(src) > 5000
    c = bshot_py.Context(0)
    try:
        for s2 in ((src,) if big else (src, src[:64], src[:3])):
            T, it = c.icp(s2, tgt)
            Tr, itr = orc.icp(s2, tgt)
            assert it == itr
            np.testing.assert_array_equal(T.view(np.uint32), Tr.view(np.uint32))
        bad = src.copy()
        bad[5] = np.nan
        T, it = c.icp(bad, tgt)
        Tr, itr = orc.icp(bad, tgt)
        assert it == itr
        # a NaN source spreads NaN through the host Umeyama: same NaN pattern (payloads may differ)
        assert np.array_equal(np.isnan(T), np.isnan(Tr))
        ok = ~np.isnan(T)
        np.testing.assert_array_equal(T[ok].view(np.uint32), Tr[ok].view(np.uint32))
    finally:
        c.close()


def test_icp_target_beyond_grid_range_fails_loudly():
    """A11: a finite target beyond the target grids' key range (2^20 cells of 500 mm, about +-524 km)
    is in no cell: the ICP call fails with BSHOT_ECAP instead of matching against the other targets;
    the same context then runs an in-range call normally (the flag is per build)."""
    rng = np.random.default_rng(12)
    tgt = (rng.random((2000, 3)) * [40000, 40000, 4000] - [20000, 20000, 2000]).astype(np.float32)
    src = (tgt[:500] + rng.normal(0, 200, (500, 3))).astype(np.float32)
    far = tgt.copy()
    far[33] = (6.0e8, 0.0, 0.0)
    c = bshot_py.Context(0)
    try:
        with pytest.raises(bshot_py.BshotError, match="coordinate range"):
            c.icp(src, far)
        T, it = c.icp(src, tgt)
        Tr, itr = orc.icp(src, tgt)
        assert it == itr
        np.testing.assert_array_equal(T.view(np.uint32), Tr.view(np.uint32))
    finally:
        c.close()


@pytest.mark.parametrize("seed,frac", [(1, 0.6), (2, 0.3), (3, 0.9), (4, 0.05), (6, 0.15)])
def test_ransac_dev_matches_host(ctx, seed, frac):
    """A10 with the hypotheses scored on the GPU (bshot_ransac_dev) == host RANSAC == oracle, bit
    for bit."""
    from test_host import _corr_set
    src, tgt, cq, cm = _corr_set(seed, inlier_frac=frac)
    rc, T, iq, im = ctx.ransac(src, tgt, cq, cm)
    hrc, hT, hq, hm = bshot_py.ransac(src, tgt, cq, cm)
    orc_rc, oT, oq, om = orc.ransac(src, tgt, cq, cm)
    assert rc == hrc == orc_rc
    assert np.array_equal(T.view(np.uint32), hT.view(np.uint32))
    assert np.array_equal(T.view(np.uint32), oT.view(np.uint32))
    assert np.array_equal(iq, oq) and np.array_equal(im, om)
    for ncorr in (0, 2, 3):
        r2 = ctx.ransac(src, tgt, cq[:ncorr], cm[:ncorr])
        o2 = orc.ransac(src, tgt, cq[:ncorr], cm[:ncorr])
        assert r2[0] == o2[0] and np.array_equal(r2[1], o2[1]) and np.array_equal(r2[2], o2[2])


@pytest.mark.parametrize("nidx,nhyp", [(1, 1), (3, 63), (5, 64), (600, 65), (601, 2001), (2048, 130)])
def test_ransac_scores_kernel(ctx, nidx, nhyp):
    """k_ransac_score (workgroup per 64 hypotheses, lane per model, waves over correspondence
    quarters) == the host scorer bshot_ransac uses, count for count, including workgroups with
    fewer hypotheses than lanes and waves whose correspondence quarter is empty."""
    from test_host import _corr_set
    src, tgt, cq, cm = _corr_set(nidx + 7, n_src=max(nidx, 3), n_corr=nidx, inlier_frac=0.5)
    cs, ct = src[cq], tgt[cm]
    rng = np.random.default_rng(nhyp)
    hyp = rng.integers(0, nidx, (nhyp, 3)).astype(np.int32)
    g = bshot_py.ransac_scores(cs, ct, hyp, ctx=ctx)
    h = bshot_py.ransac_scores(cs, ct, hyp)
    assert np.array_equal(g, h)
    assert g.min() >= 0 and g.max() <= nidx


@pytest.mark.parametrize("rank_wg,rank_max,slices", [(0, -1, 1), (1, -1, 1), (1, 0, 1), (1, 1 << 30, 1), (1, -1, 3),
                                                     (0, -1, 7)])
def test_describe_rank_kernels_agree(ctx, cloud, sr_ref, rank_wg, rank_max, slices):
    """The two SHOT rank kernels (a wave per 64-rank chunk; a workgroup per keypoint staging
    whole-bucket spans in LDS, each span ranked in place or bitonic-sorted: rank_max 0 sorts every
    span, 2^30 ranks every span in place) give the host-planned describe's bits and histograms
    exactly, on the device plan and on the host plan; so do the histogram and rank_wg kernels
    launched in LPT slices (option desc_slices)."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 2048)
    kps = cloud[kidx]
    ctx.set_cloud(cloud)
    ctx.set_option("rank_wg", 0)
    ctx.set_option("dev_plan_hint", 0)
    ref_bits, ref_shot, _ = ctx.describe(kps)
    ctx.set_option("rank_wg", rank_wg)
    ctx.set_option("rank_max", rank_max)
    ctx.set_option("desc_slices", slices)
    try:
        for hint in (0, 1 << 30):
            ctx.set_option("dev_plan_hint", hint)
            bits, shot, _ = ctx.describe(kps)
            np.testing.assert_array_equal(bits, ref_bits)
            np.testing.assert_array_equal(shot.view(np.uint32), ref_shot.view(np.uint32))
    finally:
        ctx.set_option("rank_wg", 2)
        ctx.set_option("rank_max", -1)
        ctx.set_option("desc_slices", 1)


def test_lds_lane_order_check(ctx):
    """The packed SHOT apply (12 ranks per LDS float atomic) relies on same-address lanes of one
    ds_add_f32 being applied in ascending lane order; the device check behind it must find no
    mismatch, have real power (bins where the descending order differs), and leave the packed
    apply active on this device."""
    mism, sens, active = ctx.lds_lane_order()
    assert mism == 0
    assert sens > 1000
    assert active


def test_hist_pack_matches_one_rank_apply(ctx, cloud, sr_ref):
    """The packed apply and the one-rank-per-instruction apply give the same histograms and bits,
    bit for bit, and both equal the oracle (test_describe_parity covers the default)."""
    ridx, rrat = sr_ref
    kidx, _ = orc.select_topk(ridx, rrat, 2048)
    kps = cloud[kidx]
    ctx.set_cloud(cloud)
    bits1, shot1, _ = ctx.describe(kps)
    ctx.set_option("hist_pack", 0)
    try:
        bits0, shot0, _ = ctx.describe(kps)
    finally:
        ctx.set_option("hist_pack", 1)
    np.testing.assert_array_equal(bits1, bits0)
    np.testing.assert_array_equal(shot1.view(np.uint32), shot0.view(np.uint32))


def test_config5_dense_large_radius_describe():
    """BASELINE config 5: VLP-128-style 256k-point sweep, K=4096 keypoints, SHOT radius 5000 mm
    (the large-neighbourhood stress case). The GPU describes all 4096 keypoints and the oracle
    checks every one of them against the same persistent normals array, bit for bit (a few seconds
    of OpenMP on the host)."""
    pc, _ = bshot_py.synth_sweep(2, sensor=1)
    prm = bshot_py.default_params(num_keypoints=4096, shot_radius=5000.0)
    c = bshot_py.Context(0, prm)
    try:
        c.set_cloud(pc)
        idx, rat = c.seg_ratio()
        kidx, _ = bshot_py.select_topk(idx, rat, 4096)
        kps = pc[kidx]
        bits, shot, rf = c.describe(kps)
    finally:
        c.close()
    assert len(pc) > 200000 and len(kps) == 4096
    # the CV SR of the whole 245k-point sweep against the oracle's (the keypoints
    # above come from the GPU's own SR), on all host cores
    orc.set_point_threads(min(16, os.cpu_count() or 1))
    try:
        ridx, rrat = orc.seg_ratio(pc)
    finally:
        orc.set_point_threads(1)
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(rat.view(np.uint32), rrat.view(np.uint32))
    rn = orc.normals(pc, kps)
    rs, rrf = orc.shot(pc, rn, kps, radius=5000.0)
    np.testing.assert_array_equal(shot.view(np.uint32), rs.view(np.uint32))
    np.testing.assert_array_equal(rf.view(np.uint32), rrf.view(np.uint32))
    np.testing.assert_array_equal(bits, orc.binarize(rs))
