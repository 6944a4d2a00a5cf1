"""Preprocessor (reference src/preprocess.cpp:38-227) -- CPU tier.

The reference ships no fixture for this stage, so the C++ oracle (oracle/oracle_pre.cpp, std::map
restatement) is cross-checked here against a second, independent pure-Python restatement of the
same file (sorted dicts, CPython's libm = glibc, numpy float32 for the Eigen::Vector3f points) on
small adversarial inputs: shuffled records, duplicate keys (last write wins), lost points,
+-0 verticals, selection lists, vert_init inside the vertical range, vertical tables that miss
the data (operator[] insertions). Parity vs the reference binary: unpinned (it cannot be built)."""
import math

import numpy as np
import pytest

import bshot_py
import oracle_ref as orc

PI = 3.1415926535897932384626433832795
f32 = np.float32


def _norm(p):
    return f32(math.sqrt(f32(f32(p[0] * p[0]) + f32(p[1] * p[1])) + f32(p[2] * p[2])))


def _v3(x, y, z):
    return (f32(x), f32(y), f32(z))


def _sub(a, b):
    return (f32(a[0] - b[0]), f32(a[1] - b[1]), f32(a[2] - b[2]))


class _OrderedMap(dict):
    """std::map<double, .> stand-in: keys compare as doubles (+0 == -0 keeps the first key)."""

    def _find(self, k):
        for kk in self.keys():
            if kk == k:
                return kk
        return None

    def set(self, k, v):
        kk = self._find(k)
        self[k if kk is None else kk] = v

    def get_ins(self, k, default):  # operator[]
        kk = self._find(k)
        if kk is None:
            self[k] = default
            return default
        return self[kk]

    def items_sorted(self):
        return sorted(self.items(), key=lambda kv: kv[0])


def py_preprocess(L, vert_deg, vert_init, lowpt_th, sel=None, save_sel=True):
    rimg, rmmap, selmap = _OrderedMap(), _OrderedMap(), _OrderedMap()

    def inner(m, k):
        kk = m._find(k)
        if kk is None:
            m[k] = _OrderedMap()
            return m[k]
        return m[kk]

    selpts = sorted(sel) if sel is not None else []
    selidx = 0
    for i, l in enumerate(L):
        dist = float(l["distance"]) * 2
        az = float(l["azimuth"]) * PI / 180.0
        vr = float(l["vertical"]) * PI / 180.0
        inner(rimg, az).set(vr, dist)
        inner(rimg, az).set(vert_init, 2450 / math.sin(vert_init))
        inner(rmmap, az).set(vr, 0)
        inner(rmmap, az).set(vert_init, 1)
        if sel is None:
            inner(selmap, az).set(vr, True)
        elif selidx < len(selpts) and selpts[selidx] == i:
            inner(selmap, az).set(vr, True)
            selidx += 1
        else:
            inner(selmap, az).set(vr, False)
    grad_th, height_th, dist_th, angdiff = 45.0, 500.0, 3000.0, 1.0 * PI / 180.0
    for az, col in rimg.items_sorted():
        rm = inner(rmmap, az)
        first, lost, set_th, prev_g = True, False, False, True
        r0 = -2450 / math.tan(vert_init)
        p_prev = _v3(r0 * math.sin(az), r0 * math.cos(az), -2450.0)
        p_th = p_prev
        for vr, d in col.items_sorted():
            if first:
                first = False
                continue
            x = d * math.cos(vr) * math.sin(az)
            y = d * math.cos(vr) * math.cos(az)
            z = d * math.sin(vr)
            pc = _v3(x, y, z)
            with np.errstate(invalid="ignore", divide="ignore"):
                q = f32(f32(pc[2] - p_prev[2]) / _norm(_sub(pc, p_prev)))
                a = f32(np.arcsin(q))
            grad = float(f32(a * f32(180))) / PI
            pn = float(_norm(p_prev))
            if prev_g and (grad > grad_th or d == 0 or d < pn):
                set_th, p_th = True, p_prev
            if prev_g:
                if grad < grad_th and not lost:
                    rm.set(vr, 1)
                else:
                    rm.set(vr, 0)
                    prev_g = False
            elif float(pc[2]) < lowpt_th and grad < grad_th:
                rm.set(vr, 1)
                prev_g, set_th = True, False
            if d == 0:
                rm.set(vr, 1)
                lost, prev_g = True, False
            else:
                lost = False
            if d < pn and d != 0:
                rm.set(vr, 0)
                prev_g = False
            if set_th and float(f32(pc[2] - p_th[2])) < height_th and pc[2] < p_prev[2]:
                set_th = False
                rm.set(vr, 1)
                prev_g = True
            if -820 <= x <= 820 and -1800 <= y <= 1300 and -2000 <= z <= 100:
                rm.set(vr, 2)
            p_prev = pc
    for vdeg in sorted(vert_deg):
        v = vdeg * PI / 180.0
        prev_hor, first = None, True
        for az, _ in rimg.items_sorted():
            if first:
                prev_hor, first = az, False
            elif inner(rimg, az).get_ins(v, 0.0) == 0:
                continue
            else:
                dd = inner(rimg, az).get_ins(v, 0.0) - inner(rimg, prev_hor).get_ins(v, 0.0)
                dh = az - prev_hor
                if abs(dd) > dist_th and abs(dh) < angdiff:
                    tgt = az if dd > 0 else prev_hor
                    if inner(rmmap, tgt).get_ins(v, 0) == 0:
                        inner(rmmap, tgt).set(v, 3)
                prev_hor = az
    cells = []
    for az, col in rimg.items_sorted():
        for vr, d in col.items_sorted():
            rmv = inner(rmmap, az)._find(vr)
            slv = inner(selmap, az)._find(vr)
            cells.append((az, vr, d, inner(rmmap, az)[rmv] if rmv is not None else -1,
                          int(inner(selmap, az)[slv]) if slv is not None else -1))
    pts = []
    for az, vr, d, rmv, slv in cells:
        if d == 0 or vr == vert_init:
            continue
        if rmv == 0 and slv == int(save_sel):
            pts.append(_v3(d * math.cos(vr) * math.sin(az), d * math.cos(vr) * math.cos(az), d * math.sin(vr)))
    return np.array(pts, np.float32).reshape(-1, 3), cells


def _small_case(seed, ncol=6, nv=8, dup=True, shuffle=True):
    rng = np.random.default_rng(seed)
    verts = sorted(rng.uniform(-30, 10, nv).round(2).tolist())
    verts[0] = 0.0 if seed % 3 == 0 else verts[0]
    recs = []
    for c in range(ncol):
        az = round(c * 0.4 + (0.05 if seed % 2 else 0.0), 2)
        for v in verts:
            d = int(rng.integers(500, 20000)) if rng.random() > 0.15 else 0
            recs.append((az, v, d))
    if dup:
        for _ in range(4):
            az, v, _d = recs[int(rng.integers(len(recs)))]
            recs.append((az, -0.0 if v == 0.0 else v, int(rng.integers(0, 20000))))
    if shuffle:
        rng.shuffle(recs)
    L = np.zeros(len(recs), bshot_py.LASER_DTYPE)
    for i, (az, v, d) in enumerate(recs):
        L[i]["azimuth"], L[i]["vertical"], L[i]["distance"] = az, v, d
    return L, verts


def _cells_equal(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert np.float64(x[0]).tobytes() == np.float64(y[0]).tobytes()
        assert np.float64(x[1]).tobytes() == np.float64(y[1]).tobytes()
        assert np.float64(x[2]).tobytes() == np.float64(y[2]).tobytes()
        assert int(x[3]) == int(y[3]) and int(x[4]) == int(y[4])


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("vert_init", [-0.6, -0.3])
def test_oracle_matches_python_restatement(seed, vert_init):
    L, verts = _small_case(seed)
    vlist = verts if seed % 4 else verts[:-2] + [verts[-1] + 0.5]  # a table that misses the data
    sel = None if seed % 2 else sorted(np.random.default_rng(seed).choice(len(L), len(L) // 2, replace=False))
    save = bool(seed % 3)
    for lowpt in (-1950.0, -100.0):
        xo, co = orc.preprocess(L, vlist, vert_init, lowpt, sel, save)
        xp, cp = py_preprocess(L, vlist, vert_init, lowpt, sel, save)
        np.testing.assert_array_equal(xo.view(np.uint32), xp.view(np.uint32))
        _cells_equal([tuple(r) for r in co], cp)


def test_oracle_synthetic_hdl32_sanity():
    L = bshot_py.synth_lasers(0, sensor=2)
    assert len(L) == 32 * 2170
    xyz, cells = orc.preprocess(L, bshot_py.sensor_vertical_angles(2), -0.6, -1950.0)
    codes = np.bincount(cells["rm"] + 1, minlength=5)
    # every code occurs: kept, ground/lost/vert_init, self-car (lost points sit at the origin), occluded
    assert codes[1] == len(xyz) and codes[2] > 0 and codes[3] > 0 and codes[4] > 0
    # map order: azimuth, then vertical ascending
    key = np.lexsort((cells["vertical"], cells["azimuth"]))
    assert np.array_equal(key, np.arange(len(cells)))


def test_oracle_empty_and_single():
    L = np.zeros(0, bshot_py.LASER_DTYPE)
    xyz, cells = orc.preprocess(L, [0.0])
    assert len(xyz) == 0 and len(cells) == 0
    L = np.zeros(1, bshot_py.LASER_DTYPE)
    L[0]["azimuth"], L[0]["vertical"], L[0]["distance"] = 10.0, -5.0, 4000
    xyz, cells = orc.preprocess(L, [-5.0])
    xp, cp = py_preprocess(L, [-5.0], -0.6, -2000.0)
    np.testing.assert_array_equal(xyz, xp)
    _cells_equal([tuple(r) for r in cells], cp)
