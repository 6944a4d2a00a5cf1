"""ctypes wrapper of the CPU restatement (oracle/). TEST INFRASTRUCTURE ONLY: imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the product.
PARITY UNPINNED vs PCL: see oracle/oracle_core.h."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# ORACLE_LIB: an alternative build of the restatement (the sanitizer build, oracle/Makefile sanitize)
ORACLE_LIB = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "liboracle.so")
P = ctypes.c_void_p


class OParams(ctypes.Structure):
    _fields_ = [
        ("seg_radius", ctypes.c_float), ("seg_max_nn", ctypes.c_int), ("sr_type", ctypes.c_int),
        ("num_keypoints", ctypes.c_int), ("iss_salient", ctypes.c_float), ("iss_nonmax", ctypes.c_float),
        ("iss_gamma21", ctypes.c_double), ("iss_gamma32", ctypes.c_double), ("iss_min_nn", ctypes.c_int),
        ("normal_radius", ctypes.c_float), ("normal_max_nn", ctypes.c_int), ("shot_radius", ctypes.c_float),
        ("map_range", ctypes.c_float), ("ransac_max_iter", ctypes.c_int), ("ransac_thresh", ctypes.c_double),
        ("icp_max_iter", ctypes.c_int), ("run_icp", ctypes.c_int), ("run_iss", ctypes.c_int),
        ("map_canonical", ctypes.c_int), ("eval_icp", ctypes.c_int),
    ]


class OStats(ctypes.Structure):
    _fields_ = [
        ("n_points", ctypes.c_int), ("n_valid_ratios", ctypes.c_int), ("n_keypoints", ctypes.c_int),
        ("n_iss", ctypes.c_int), ("n_target", ctypes.c_int), ("n_mutual", ctypes.c_int),
        ("n_inliers", ctypes.c_int), ("icp_iters", ctypes.c_int), ("gated", ctypes.c_int),
        ("h_diff", ctypes.c_float), ("t_diff", ctypes.c_float), ("T_ransac", ctypes.c_float * 16),
        ("pose", ctypes.c_float * 16), ("map_size", ctypes.c_int), ("repeat_sr", ctypes.c_float),
        ("repeat_iss", ctypes.c_float),
        ("corr_n", ctypes.c_int), ("corr_avg", ctypes.c_float), ("corr_sd", ctypes.c_float),
        ("corr_med", ctypes.c_float),
    ]


_L = None


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _L
    if _L is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        _L = ctypes.CDLL(ORACLE_LIB)
    return _L


def _p(a):
    return a.ctypes.data_as(P)


def params(**kw):
    p = OParams()
    lib().oracle_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def seg_ratio(xyz, radius=3000.0, max_nn=300, sr_type=0):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    n = len(xyz)
    idx = np.zeros(max(n, 1), np.int32)
    rat = np.zeros(max(n, 1), np.float32)
    m = ctypes.c_int()
    lib().oracle_seg_ratio(_p(xyz), n, ctypes.c_float(radius), max_nn, sr_type, _p(idx), _p(rat), ctypes.byref(m))
    return idx[: m.value].copy(), rat[: m.value].copy()


def select_topk(idx, ratio, k):
    idx = np.ascontiguousarray(idx, np.int32)
    ratio = np.ascontiguousarray(ratio, np.float32)
    o = np.zeros(max(k, 1), np.int32)
    r = np.zeros(max(k, 1), np.float32)
    m = ctypes.c_int()
    lib().oracle_select_keypoints(_p(idx), _p(ratio), len(idx), k, _p(o), _p(r), ctypes.byref(m))
    return o[: m.value].copy(), r[: m.value].copy()


def iss(xyz, salient=60.0, nonmax=40.0, g21=0.975, g32=0.975, min_nn=5):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    n = len(xyz)
    out = np.zeros(max(n, 1), np.int32)
    third = np.zeros(max(n, 1), np.float64)
    m = ctypes.c_int()
    lib().oracle_iss(_p(xyz), n, ctypes.c_float(salient), ctypes.c_float(nonmax), ctypes.c_double(g21),
                     ctypes.c_double(g32), min_nn, _p(out), n, ctypes.byref(m), _p(third))
    return out[: m.value].copy(), third[:n].copy()


def normals(xyz, kps, radius=3000.0, max_nn=300, prev=None):
    """Persistent-array semantics: slots [0, K) <- keypoint normals, others zero (or `prev`)."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    kps = np.ascontiguousarray(kps, np.float32).reshape(-1, 3)
    n = len(xyz)
    out = np.zeros((max(n, 1), 4), np.float32)
    if prev is not None:
        m = min(len(prev), n)
        out[:m] = prev[:m]
    lib().oracle_normals(_p(xyz), n, _p(kps), len(kps), ctypes.c_float(radius), max_nn, _p(out))
    return out[:n]


def shot(xyz, normals_arr, kps, radius=3000.0):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    kps = np.ascontiguousarray(kps, np.float32).reshape(-1, 3)
    nrm = np.ascontiguousarray(normals_arr, np.float32).reshape(-1, 4)
    k = len(kps)
    s = np.zeros((max(k, 1), 352), np.float32)
    rf = np.zeros((max(k, 1), 9), np.float32)
    lib().oracle_shot(_p(xyz), len(xyz), _p(nrm), _p(kps), k, ctypes.c_float(radius), _p(s), _p(rf))
    return s[:k], rf[:k]


def binarize(shot_arr):
    shot_arr = np.ascontiguousarray(shot_arr, np.float32).reshape(-1, 352)
    k = len(shot_arr)
    bits = np.zeros((max(k, 1), 11), np.uint32)
    lib().oracle_binarize(_p(shot_arr), k, _p(bits))
    return bits[:k]


def match(a, b):
    a = np.ascontiguousarray(a, np.uint32).reshape(-1, 11)
    b = np.ascontiguousarray(b, np.uint32).reshape(-1, 11)
    na, nb = len(a), len(b)
    left = np.zeros(max(na, 1), np.int32)
    right = np.zeros(max(nb, 1), np.int32)
    cq = np.zeros(max(na, 1), np.int32)
    cm = np.zeros(max(na, 1), np.int32)
    nc = ctypes.c_int()
    lib().oracle_match(_p(a), na, _p(b), nb, _p(left), _p(right), _p(cq), _p(cm), ctypes.byref(nc))
    return left[:na], right[:nb], cq[: nc.value], cm[: nc.value]


def ransac(src, tgt, cq, cm, max_iter=2000, thresh=1500.0):
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
    tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
    cq = np.ascontiguousarray(cq, np.int32)
    cm = np.ascontiguousarray(cm, np.int32)
    T = np.zeros(16, np.float32)
    iq = np.zeros(max(len(cq), 1), np.int32)
    im = np.zeros(max(len(cq), 1), np.int32)
    ni = ctypes.c_int()
    rc = lib().oracle_ransac(_p(src), len(src), _p(tgt), len(tgt), _p(cq), _p(cm), len(cq), max_iter,
                             ctypes.c_double(thresh), _p(T), _p(iq), _p(im), ctypes.byref(ni))
    return rc, T.reshape(4, 4), iq[: ni.value].copy(), im[: ni.value].copy()


def icp(src, tgt, max_iter=10):
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
    tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
    T = np.zeros(16, np.float32)
    it = ctypes.c_int()
    lib().oracle_icp(_p(src), len(src), _p(tgt), len(tgt), max_iter, _p(T), ctypes.byref(it))
    return T.reshape(4, 4), it.value


class Odometry:
    def __init__(self, p=None):
        self.p = p if p is not None else params()
        lib().oracle_odom_create.restype = P
        self.h = P(lib().oracle_odom_create(ctypes.byref(self.p)))

    def __del__(self):
        try:
            lib().oracle_odom_destroy(self.h)
        except Exception:
            pass

    def process(self, xyz):
        xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
        st = OStats()
        lib().oracle_odom_process(self.h, _p(xyz), len(xyz), ctypes.byref(st))
        return st

    def _get(self, fn, cols, dtype, cap=1 << 20):
        buf = np.zeros((cap, cols), dtype)
        n = fn(self.h, _p(buf), cap)
        if n < 0:
            return self._get(fn, cols, dtype, -n)
        return buf[:n].copy()

    def keypoints(self):
        return self._get(lib().oracle_odom_get_keypoints, 3, np.float32)

    def ratios(self):
        return self._get(lib().oracle_odom_get_ratios, 1, np.float32)[:, 0]

    def bits(self):
        return self._get(lib().oracle_odom_get_bits, 11, np.uint32)

    def iss(self):
        return self._get(lib().oracle_odom_get_iss, 3, np.float32)

    def target(self, cap=1 << 20):
        xyz = np.zeros((cap, 3), np.float32)
        bits = np.zeros((cap, 11), np.uint32)
        n = lib().oracle_odom_get_target(self.h, _p(xyz), _p(bits), cap)
        if n < 0:
            return self.target(-n)
        return xyz[:n].copy(), bits[:n].copy()

    def inliers(self, cap=1 << 16):
        q = np.zeros(cap, np.int32)
        m = np.zeros(cap, np.int32)
        n = lib().oracle_odom_get_inliers(self.h, _p(q), _p(m), cap)
        if n < 0:
            return self.inliers(-n)
        return q[:n].copy(), m[:n].copy()


def radius_search(xyz, q, radius, max_nn=0, cap=1 << 20):
    """Exact radius search with FLANN semantics: d2 = ((dx*dx+dy*dy)+dz*dz) in float, d2 < r^2,
    sorted by (d2, idx); max_nn > 0 keeps the max_nn nearest."""
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(q, np.float32).reshape(3)
    idx = np.zeros(cap, np.int32)
    d2 = np.zeros(cap, np.float32)
    m = lib().oracle_radius_search(_p(xyz), len(xyz), _p(q), ctypes.c_float(radius), max_nn, _p(idx), _p(d2), cap)
    return idx[:m].copy(), d2[:m].copy()


def eig3(a):
    a = np.ascontiguousarray(a, np.float64).reshape(9)
    w = np.zeros(3, np.float64)
    v = np.zeros(9, np.float64)
    lib().oracle_eig3(_p(a), _p(w), _p(v))
    return w, v.reshape(3, 3)


def umeyama(src, dst, use_float=False):
    src = np.ascontiguousarray(src, np.float64).reshape(-1, 3)
    dst = np.ascontiguousarray(dst, np.float64).reshape(-1, 3)
    T = np.zeros(16, np.float64)
    lib().oracle_umeyama(_p(src), _p(dst), len(src), int(use_float), _p(T))
    return T.reshape(4, 4)


def set_threads(n):
    """OpenMP threads for the oracle's normals/SHOT stages (the reference's OpenMP stages)."""
    lib().oracle_set_threads(int(n))
    return lib().oracle_get_threads()


def set_point_threads(n):
    """Threads for the oracle's per-point SR/ISS loops (default 1, as the reference). Used by the
    golden generator only; results do not depend on it."""
    lib().oracle_set_point_threads(int(n))


# ---- preprocessor (oracle/oracle_pre.cpp; reference src/preprocess.cpp) ----------------------------
class OPreParams(ctypes.Structure):
    _fields_ = [("vert_init", ctypes.c_double), ("lowpt_th", ctypes.c_double), ("have_sel_list", ctypes.c_int),
                ("save_sel", ctypes.c_int)]


def preprocess(lasers, vert_deg, vert_init=-0.6, lowpt_th=-2000.0, sel=None, save_sel=True):
    """Preprocessor::run restated with the reference's std::maps. Returns (xyz, cells): cells is the
    rimg table after run() with rmmap / selmap values (-1 where those maps lack the key)."""
    import bshot_py
    lasers = np.ascontiguousarray(lasers, dtype=bshot_py.LASER_DTYPE)
    vd = np.ascontiguousarray(vert_deg, dtype=np.float64)
    pp = OPreParams(vert_init, lowpt_th, 1 if sel is not None else 0, 1 if save_sel else 0)
    sa = np.ascontiguousarray(sel if sel is not None else np.zeros(0), dtype=np.int32)
    n = len(lasers)
    out = np.zeros((max(n, 1), 3), np.float32)
    m = ctypes.c_int()
    nc = ctypes.c_int()
    ccap = 2 * n + 64 * (len(vd) + 1) * (n + 1) // 32 + 1024
    cells = np.zeros(ccap, bshot_py.CELL_DTYPE)
    rc = lib().oracle_preprocess(_p(lasers), n, _p(vd), len(vd), ctypes.byref(pp), _p(sa), len(sa), _p(out), n,
                                 ctypes.byref(m), _p(cells), ccap, ctypes.byref(nc))
    if rc < 0:
        raise RuntimeError(f"oracle_preprocess capacity ({rc})")
    return out[: m.value].copy(), cells[: nc.value].copy()


# ---- Velodyne packet decode (oracle/oracle_velo.cpp; reference include/VelodyneCapture.h:413-525) ----
def velodyne_decode(payloads, unixtime, max_lasers=32, specified_frame=0):
    """capturePCAP's loop: returns (records of the pushed rotations back to back, rot_count)."""
    import bshot_py
    pk = np.ascontiguousarray(payloads, dtype=np.uint8).reshape(-1, 1206)
    ut = np.ascontiguousarray(unixtime, dtype=np.int64)
    npk = len(pk)
    out = np.zeros(max(npk * 384, 1), bshot_py.LASER_DTYPE)
    rc = np.zeros(npk * 384 + 2, np.int32)
    no, nr = ctypes.c_int(), ctypes.c_int()
    r = lib().oracle_velodyne_decode(_p(pk), _p(ut), npk, max_lasers, specified_frame, _p(out), len(out), _p(rc),
                                     len(rc), ctypes.byref(no), ctypes.byref(nr))
    if r == -1:
        raise ValueError("sensor type")
    if r < 0:
        raise RuntimeError("oracle_velodyne_decode capacity")
    out = out[: no.value].copy()
    out.view(np.uint8).reshape(-1, 32)[:, 20:24] = 0  # struct padding (indeterminate in the reference too)
    return out, rc[: nr.value].copy()
