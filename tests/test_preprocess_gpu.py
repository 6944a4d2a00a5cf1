"""Preprocessor on the GPU (csrc/preprocess.hip) vs the oracle (oracle/oracle_pre.cpp), same inputs.

Bit-exact tier: output points (float32 bits, count and map order) and the whole range image as
getRangeImage / getRemoveMap / getSelMap return it (keys and ranges as float64 bits, removal codes,
selection flags). Per-point sin/cos/asin run in the device's libm and the oracle's glibc; a
difference could only surface if a 1-ulp libm difference survived the rounding to float32 or sat on
a threshold -- the tests assert exact equality on every case below."""
import numpy as np
import pytest

import bshot_py
import oracle_ref as orc
from test_preprocess import _small_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = bshot_py.Context(0)
    yield c
    c.close()


def _check(ctx, L, vlist, vert_init=-0.6, lowpt=-1950.0, sel=None, save=True):
    g = ctx.preprocess(L, vlist, vert_init, lowpt, sel, save)
    gc = ctx.preprocess_cells()
    r, rc = orc.preprocess(L, vlist, vert_init, lowpt, sel, save)
    assert g.shape == r.shape
    np.testing.assert_array_equal(g.view(np.uint32), r.view(np.uint32))
    assert len(gc) == len(rc)
    for f in ("azimuth", "vertical", "distance"):
        np.testing.assert_array_equal(gc[f].view(np.uint64), rc[f].view(np.uint64), err_msg=f)
    np.testing.assert_array_equal(gc["rm"], rc["rm"])
    np.testing.assert_array_equal(gc["sel"], rc["sel"])
    return g


@pytest.mark.parametrize("fast", [1, 0])
@pytest.mark.parametrize("sensor,frame", [(2, 0), (2, 7), (0, 0), (1, 3)])
def test_synthetic_rotation_exact(ctx, sensor, frame, fast):
    """Azimuth-ordered rotations with tabled verticals take the one-sort fast path (fast=1); the
    general two-sort path (knob pre_fast=0) must give the same bits."""
    ctx.set_option("pre_fast", fast)
    L = bshot_py.synth_lasers(frame, sensor=sensor)
    g = _check(ctx, L, bshot_py.sensor_vertical_angles(sensor))
    assert len(g) > 10000
    ctx.set_option("pre_fast", 1)


def test_shuffled_with_duplicates_and_selection(ctx):
    L = bshot_py.synth_lasers(2, sensor=2)
    rng = np.random.default_rng(5)
    extra = L[rng.integers(0, len(L), 3000)].copy()
    extra["distance"] = rng.integers(0, 30000, len(extra))
    L2 = np.concatenate([L, extra])
    L2 = L2[rng.permutation(len(L2))]
    v = bshot_py.sensor_vertical_angles(2)
    _check(ctx, L2, v)
    sel = np.sort(rng.choice(len(L2), len(L2) // 3, replace=False))
    _check(ctx, L2, v, sel=sel, save=True)
    _check(ctx, L2, v, sel=sel, save=False)
    _check(ctx, L2, v, vert_init=-0.3, lowpt=-1450.0)  # vert_init inside the vertical range


@pytest.mark.parametrize("seed", range(6))
def test_small_adversarial_exact(ctx, seed):
    L, verts = _small_case(seed)
    vlist = verts if seed % 4 else verts[:-2] + [verts[-1] + 0.5]
    _check(ctx, L, vlist, vert_init=-0.6 if seed % 2 else -0.3, lowpt=-100.0)
    _check(ctx, L, vlist + [-0.6 * 180.0 / 3.1415926535897932384626433832795])  # vert_init in the table


def test_empty_single_and_no_table(ctx):
    assert len(ctx.preprocess(np.zeros(0, bshot_py.LASER_DTYPE), [0.0])) == 0
    L = np.zeros(1, bshot_py.LASER_DTYPE)
    L[0]["azimuth"], L[0]["vertical"], L[0]["distance"] = 10.0, -5.0, 4000
    _check(ctx, L, [-5.0])
    _check(ctx, bshot_py.synth_lasers(1, sensor=2), [])


def test_device_path_feeds_odometry_cloud(ctx):
    import torch
    L = bshot_py.synth_lasers(4, sensor=0)
    v = bshot_py.sensor_vertical_angles(0)
    dl = torch.from_numpy(L.view(np.uint8)).cuda()
    out = torch.zeros((len(L), 3), dtype=torch.float32, device="cuda")
    n = ctx.preprocess_device(dl.data_ptr(), len(L), v, out.data_ptr(), len(L), lowpt_th=-1950.0)
    r, _ = orc.preprocess(L, v, -0.6, -1950.0)
    assert n == len(r)
    np.testing.assert_array_equal(out[:n].cpu().numpy().view(np.uint32), r.view(np.uint32))
