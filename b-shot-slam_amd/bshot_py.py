"""ctypes binding of libbshot_amd.so (the C ABI in include/bshot_abi.h) for tests and bench.py.

This is a thin host-side mirror of the reference's LidarOdometry frame loop
(test/odometry_test.cpp:159-194) over the C ABI; every compute call runs the gfx950 kernels.
The product never falls back to CPU: a missing library or GPU raises.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BSHOT_LIB: diagnostic override (timing experiments on `make variant` builds)
LIB_PATH = os.environ.get("BSHOT_LIB") or os.path.join(HERE, "lib", "libbshot_amd.so")
SYNTH_PATH = os.path.join(HERE, "lib", "libbshot_synth.so")
P = ctypes.c_void_p

NSTAGES = 12
STAGE_NAMES = ["grid", "seg_ratio", "iss", "normals", "shot_gather", "shot_sort", "lrf", "shot_hist", "match", "icp",
               "ransac", "preprocess"]


class Params(ctypes.Structure):
    _fields_ = [
        ("seg_radius", ctypes.c_float), ("seg_max_nn", ctypes.c_int), ("sr_type", ctypes.c_int),
        ("num_keypoints", ctypes.c_int), ("iss_salient", ctypes.c_float), ("iss_nonmax", ctypes.c_float),
        ("iss_gamma21", ctypes.c_double), ("iss_gamma32", ctypes.c_double), ("iss_min_nn", ctypes.c_int),
        ("normal_radius", ctypes.c_float), ("normal_max_nn", ctypes.c_int), ("shot_radius", ctypes.c_float),
        ("map_range", ctypes.c_float), ("ransac_max_iter", ctypes.c_int), ("ransac_thresh", ctypes.c_double),
        ("icp_max_iter", ctypes.c_int), ("run_icp", ctypes.c_int), ("run_iss", ctypes.c_int),
        ("run_kp_eval", ctypes.c_int),
    ]


class FrameStats(ctypes.Structure):
    _fields_ = [
        ("n_points", ctypes.c_int), ("n_valid_ratios", ctypes.c_int), ("n_keypoints", ctypes.c_int),
        ("n_iss", ctypes.c_int), ("n_target", ctypes.c_int), ("n_mutual", ctypes.c_int),
        ("n_inliers", ctypes.c_int), ("icp_iters", ctypes.c_int), ("gated", ctypes.c_int),
        ("h_diff", ctypes.c_float), ("t_diff", ctypes.c_float), ("T_ransac", ctypes.c_float * 16),
        ("pose", ctypes.c_float * 16), ("map_size", ctypes.c_int), ("repeat_sr", ctypes.c_float),
        ("repeat_iss", ctypes.c_float), ("host_ms", ctypes.c_float * 8),
        ("corr_n", ctypes.c_int), ("corr_avg", ctypes.c_float), ("corr_sd", ctypes.c_float),
        ("corr_med", ctypes.c_float),
    ]
    HOST_PHASES = ["extract", "iss", "describe", "match", "ransac", "icp", "map", "kp_eval"]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("T_ransac", "pose", "host_ms")}
        d["host_ms"] = dict(zip(self.HOST_PHASES, list(self.host_ms)))
        d["T_ransac"] = np.array(self.T_ransac, np.float32).reshape(4, 4)
        d["pose"] = np.array(self.pose, np.float32).reshape(4, 4)
        return d


ABI_SYMBOLS = [
    "bshot_default_params", "bshot_create", "bshot_destroy", "bshot_last_error", "bshot_sync", "bshot_stream",
    "bshot_set_cloud", "bshot_set_cloud_device", "bshot_seg_ratio", "bshot_select_topk", "bshot_iss",
    "bshot_describe", "bshot_get_normals", "bshot_match", "bshot_ransac", "bshot_ransac_dev", "bshot_ransac_scores", "bshot_icp", "bshot_odom_create",
    "bshot_odom_destroy", "bshot_odom_last_error", "bshot_odom_process", "bshot_odom_process_device",
    "bshot_odom_get_keypoints", "bshot_odom_get_ratios", "bshot_odom_get_bits", "bshot_odom_get_target",
    "bshot_odom_get_inliers", "bshot_odom_get_iss", "bshot_odom_ctx", "bshot_odom_map_delta",
    "bshot_odom_replica_insert", "bshot_odom_replica_size", "bshot_stage_times", "bshot_stage_reset",
    "bshot_set_timing", "bshot_work_counters", "bshot_radius_pairs", "bshot_debug_knn_stats",
    "bshot_debug_lds_lane_order",
    "bshot_map_create", "bshot_map_destroy", "bshot_map_add", "bshot_map_query", "bshot_map_size",
    "bshot_map_set_query_mode",
    "bshot_map_block_id", "bshot_set_option", "bshot_prefetch_cloud_device", "bshot_odom_set_next_device",
    "bshot_odom_set_option", "bshot_odom_set_metrics_file", "bshot_odom_upload", "bshot_odom_drain", "bshot_xchg_unique_id", "bshot_xchg_create",
    "bshot_xchg_destroy", "bshot_odom_exchange", "bshot_odom_exchange_sim", "bshot_odom_gpu_replica_size", "bshot_odom_gpu_replica_query",
    "bshot_odom_gpu_replica_insert", "bshot_queue_cloud_device", "bshot_odom_set_next2_device",
    "bshot_pre_default_params", "bshot_preprocess", "bshot_preprocess_device", "bshot_preprocess_cells",
    "bshot_pcap_load", "bshot_velodyne_decode", "bshot_velodyne_decode_device",
    "bshot_odom_extract_device", "bshot_odom_process_record",
]

# velodyne::Laser (include/VelodyneCapture.h:43-50) == bshot_laser: 32 B, int64 time at offset 24
LASER_DTYPE = np.dtype({"names": ["azimuth", "vertical", "distance", "intensity", "id", "time"],
                        "formats": ["<f8", "<f8", "<u2", "u1", "u1", "<i8"],
                        "offsets": [0, 8, 16, 18, 19, 24], "itemsize": 32})
# bshot_pre_cell: one getRangeImage entry with its getRemoveMap / getSelMap values (-1: no entry)
CELL_DTYPE = np.dtype([("azimuth", "<f8"), ("vertical", "<f8"), ("distance", "<f8"), ("rm", "<i4"), ("sel", "<i4")])
# HDL-32E vertical table (include/VelodyneCapture.h:572), laser-id order
HDL32_VERTICAL = [-30.67, -9.3299999, -29.33, -8.0, -28, -6.6700001, -26.67, -5.3299999, -25.33, -4.0, -24.0,
                  -2.6700001, -22.67, -1.33, -21.33, 0.0, -20.0, 1.33, -18.67, 2.6700001, -17.33, 4.0, -16,
                  5.3299999, -14.67, 6.6700001, -13.33, 8.0, -12.0, 9.3299999, -10.67, 10.67]


class PreParams(ctypes.Structure):
    _fields_ = [("vert_init", ctypes.c_double), ("lowpt_th", ctypes.c_double), ("have_sel_list", ctypes.c_int),
                ("save_sel", ctypes.c_int)]


def pre_params(vert_init=-0.6, lowpt_th=-2000.0, have_sel_list=False, save_sel=True):
    return PreParams(vert_init, lowpt_th, 1 if have_sel_list else 0, 1 if save_sel else 0)


def sensor_vertical_angles(sensor):
    """Vertical angle table (degrees) of synth_lasers' sensors, as capture.getVerticalAngle() gives it."""
    if sensor == 0:
        return [2.0 + (-8.33 - 2.0) * i / 31.0 for i in range(32)] + \
               [-8.83 + (-24.33 + 8.83) * i / 31.0 for i in range(32)]
    if sensor == 1:
        return [-25.0 + 40.0 * i / 127.0 for i in range(128)]
    return list(HDL32_VERTICAL)

_lib = None
_synth = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libbshot_amd.so not built ({LIB_PATH}); run __graft_entry__.build()")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (soname
        # libamdhip64.so.7, loaded by torch under the name libamdhip64.so). Loaded after ours, it
        # would bring a second HIP/HSA runtime that finds no GPU; loaded first, the library binds to
        # it by soname. So torch, when installed, is imported before the library is opened.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.bshot_last_error.restype = ctypes.c_char_p
        _lib.bshot_odom_last_error.restype = ctypes.c_char_p
        _lib.bshot_stream.restype = P
        _lib.bshot_odom_ctx.restype = P
        _lib.bshot_map_create.restype = P
        _lib.bshot_map_block_id.restype = ctypes.c_uint64
    return _lib


def default_params(**kw):
    p = Params()
    lib().bshot_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _f32(a, cols=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


def _ptr(a):
    return a.ctypes.data_as(P)


class BshotError(RuntimeError):
    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


ESTALE = -5  # BSHOT_ESTALE: a frame-sharded record described over other normals than the sequence's


class Context:
    """One GPU, one HIP stream (bshot_ctx)."""

    def __init__(self, device=0, params=None):
        self.L = lib()
        self.h = P()
        self.params = params if params is not None else default_params()
        rc = self.L.bshot_create(ctypes.byref(self.h), device, ctypes.byref(self.params))
        if rc != 0:
            raise BshotError(f"bshot_create failed ({rc}): no usable GPU?")

    def _chk(self, rc, what):
        if rc < 0:
            raise BshotError(f"{what}: {self.L.bshot_last_error(self.h).decode()} ({rc})", rc)
        return rc

    def close(self):
        if self.h:
            self.L.bshot_destroy(self.h)
            self.h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_cloud(self, xyz):
        xyz = _f32(xyz).reshape(-1, 3)
        self._xyz = xyz
        self.n = len(xyz)
        self._chk(self.L.bshot_set_cloud(self.h, _ptr(xyz), self.n), "set_cloud")

    def prefetch_cloud_device(self, dptr, n):
        self._chk(self.L.bshot_prefetch_cloud_device(self.h, P(dptr), n), "prefetch_cloud_device")

    def queue_cloud_device(self, dptr, n):
        self._chk(self.L.bshot_queue_cloud_device(self.h, P(dptr), n), "queue_cloud_device")

    def set_cloud_device(self, dptr, n):
        self.n = n
        self._chk(self.L.bshot_set_cloud_device(self.h, P(dptr), n), "set_cloud_device")

    def seg_ratio(self):
        idx = np.zeros(max(self.n, 1), np.int32)
        rat = np.zeros(max(self.n, 1), np.float32)
        m = ctypes.c_int()
        self._chk(self.L.bshot_seg_ratio(self.h, _ptr(idx), _ptr(rat), ctypes.byref(m)), "seg_ratio")
        return idx[: m.value].copy(), rat[: m.value].copy()

    def iss(self):
        out = np.zeros(max(self.n, 1), np.int32)
        m = ctypes.c_int()
        self._chk(self.L.bshot_iss(self.h, _ptr(out), len(out), ctypes.byref(m)), "iss")
        return out[: m.value].copy()

    def preprocess(self, lasers, vert_deg, vert_init=-0.6, lowpt_th=-2000.0, sel=None, save_sel=True):
        """myslam::Preprocessor::run on the GPU (bshot_preprocess): laser records -> kept points."""
        lasers = np.ascontiguousarray(lasers, dtype=LASER_DTYPE)
        vd = np.ascontiguousarray(vert_deg, dtype=np.float64)
        pp = pre_params(vert_init, lowpt_th, sel is not None, save_sel)
        sa = np.ascontiguousarray(sel if sel is not None else np.zeros(0), dtype=np.int32)
        n = len(lasers)
        out = np.zeros((max(n, 1), 3), np.float32)
        m = ctypes.c_int()
        self._chk(self.L.bshot_preprocess(self.h, _ptr(lasers), n, _ptr(vd), len(vd), ctypes.byref(pp), _ptr(sa),
                                          len(sa), _ptr(out), n, ctypes.byref(m)), "preprocess")
        return out[: m.value].copy()

    def preprocess_device(self, d_lasers, n, vert_deg, d_xyz, cap, vert_init=-0.6, lowpt_th=-2000.0):
        vd = np.ascontiguousarray(vert_deg, dtype=np.float64)
        pp = pre_params(vert_init, lowpt_th)
        m = ctypes.c_int()
        self._chk(self.L.bshot_preprocess_device(self.h, P(d_lasers), n, _ptr(vd), len(vd), ctypes.byref(pp), None,
                                                 0, P(d_xyz), cap, ctypes.byref(m)), "preprocess_device")
        return m.value

    def velodyne_decode(self, payloads, unixtime, max_lasers=32, specified_frame=0):
        """VelodyneCapture's packet loop on the GPU (bshot_velodyne_decode): 1206-B packets ->
        (records of the pushed rotations back to back, rot_start, rot_count)."""
        pk = np.ascontiguousarray(payloads, dtype=np.uint8).reshape(-1, 1206)
        ut = np.ascontiguousarray(unixtime, dtype=np.int64)
        npk = len(pk)
        out = np.zeros(max(npk * 384, 1), LASER_DTYPE)
        rs = np.zeros(npk * 384 + 2, np.int32)
        rc = np.zeros(npk * 384 + 2, np.int32)
        nr, no = ctypes.c_int(), ctypes.c_int()
        self._chk(self.L.bshot_velodyne_decode(self.h, _ptr(pk), _ptr(ut), npk, max_lasers, specified_frame, _ptr(out),
                                               len(out), _ptr(rs), _ptr(rc), len(rs), ctypes.byref(nr), ctypes.byref(no)),
                  "velodyne_decode")
        return out[: no.value].copy(), rs[: nr.value].copy(), rc[: nr.value].copy()

    def velodyne_decode_device(self, d_payloads, d_unixtime, npk, d_out, max_lasers=32, specified_frame=0):
        rs = np.zeros(npk * 384 + 2, np.int32)
        rc = np.zeros(npk * 384 + 2, np.int32)
        nr = ctypes.c_int()
        self._chk(self.L.bshot_velodyne_decode_device(self.h, P(d_payloads), P(d_unixtime), npk, max_lasers,
                                                      specified_frame, P(d_out), _ptr(rs), _ptr(rc), len(rs),
                                                      ctypes.byref(nr)), "velodyne_decode_device")
        return rs[: nr.value].copy(), rc[: nr.value].copy()

    def preprocess_cells(self):
        m = ctypes.c_int()
        self.L.bshot_preprocess_cells(self.h, None, 0, ctypes.byref(m))
        out = np.zeros(max(m.value, 1), CELL_DTYPE)
        self._chk(self.L.bshot_preprocess_cells(self.h, _ptr(out), len(out), ctypes.byref(m)), "preprocess_cells")
        return out[: m.value].copy()

    def describe(self, kps, want_shot=True):
        kps = _f32(kps).reshape(-1, 3)
        k = len(kps)
        bits = np.zeros((max(k, 1), 11), np.uint32)
        shot = np.zeros((max(k, 1), 352), np.float32) if want_shot else None
        rf = np.zeros((max(k, 1), 9), np.float32) if want_shot else None
        self._chk(self.L.bshot_describe(self.h, _ptr(kps), k, _ptr(shot) if want_shot else None,
                                        _ptr(rf) if want_shot else None, _ptr(bits)), "describe")
        if want_shot:
            return bits[:k], shot[:k], rf[:k]
        return bits[:k]

    def normals(self, n):
        out = np.zeros((max(n, 1), 4), np.float32)
        self._chk(self.L.bshot_get_normals(self.h, _ptr(out), n), "get_normals")
        return out[:n]

    def match(self, a, b):
        a = np.ascontiguousarray(a, np.uint32).reshape(-1, 11)
        b = np.ascontiguousarray(b, np.uint32).reshape(-1, 11)
        na, nb = len(a), len(b)
        left = np.zeros(max(na, 1), np.int32)
        right = np.zeros(max(nb, 1), np.int32)
        cq = np.zeros(max(na, 1), np.int32)
        cm = np.zeros(max(na, 1), np.int32)
        nc = ctypes.c_int()
        self._chk(self.L.bshot_match(self.h, _ptr(a), na, _ptr(b), nb, _ptr(left), _ptr(right), _ptr(cq), _ptr(cm),
                                     ctypes.byref(nc)), "match")
        return left[:na], right[:nb], cq[: nc.value], cm[: nc.value]

    def icp(self, src, tgt, max_iter=10):
        src = _f32(src).reshape(-1, 3)
        tgt = _f32(tgt).reshape(-1, 3)
        T = np.zeros(16, np.float32)
        it = ctypes.c_int()
        self._chk(self.L.bshot_icp(self.h, _ptr(src), len(src), _ptr(tgt), len(tgt), max_iter, _ptr(T),
                                   ctypes.byref(it)), "icp")
        return T.reshape(4, 4), it.value

    def ransac(self, src, tgt, cq, cm, max_iter=2000, thresh=1500.0):
        """A10 with every hypothesis scored on the GPU (bshot_ransac_dev); same result as ransac()."""
        src = _f32(src).reshape(-1, 3)
        tgt = _f32(tgt).reshape(-1, 3)
        cq = np.ascontiguousarray(cq, np.int32)
        cm = np.ascontiguousarray(cm, np.int32)
        T = np.zeros(16, np.float32)
        iq = np.zeros(max(len(cq), 1), np.int32)
        im = np.zeros(max(len(cq), 1), np.int32)
        ni = ctypes.c_int()
        rc = self.L.bshot_ransac_dev(self.h, _ptr(src), len(src), _ptr(tgt), len(tgt), _ptr(cq), _ptr(cm), len(cq),
                                     max_iter, ctypes.c_double(thresh), _ptr(T), _ptr(iq), _ptr(im), ctypes.byref(ni))
        self._chk(rc, "ransac_dev")
        return rc, T.reshape(4, 4), iq[: ni.value].copy(), im[: ni.value].copy()

    def set_timing(self, on):
        self.L.bshot_set_timing(self.h, 1 if on else 0)

    def set_option(self, name, value):
        self._chk(self.L.bshot_set_option(self.h, name.encode(), int(value)), "set_option")

    def stage_times(self):
        ms = (ctypes.c_double * NSTAGES)()
        nl = (ctypes.c_int64 * NSTAGES)()
        self.L.bshot_stage_times(self.h, ms, nl, NSTAGES)
        return {STAGE_NAMES[i]: (ms[i], nl[i]) for i in range(NSTAGES)}

    def stage_reset(self):
        self.L.bshot_stage_reset(self.h)

    def work(self):
        w = (ctypes.c_int64 * 12)()
        self.L.bshot_work_counters(self.h, w, 12)
        return list(w)

    def sync(self):
        self._chk(self.L.bshot_sync(self.h), "sync")

    def knn_stats(self):
        w = (ctypes.c_int64 * 32)()
        self._chk(self.L.bshot_debug_knn_stats(self.h, w, 32), "knn_stats")
        return list(w)

    def lds_lane_order(self):
        m, s, a = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.L.bshot_debug_lds_lane_order(self.h, ctypes.byref(m), ctypes.byref(s), ctypes.byref(a)),
                  "lds_lane_order")
        return m.value, s.value, bool(a.value)

    def radius_pairs(self, R):
        t = ctypes.c_int64()
        self._chk(self.L.bshot_radius_pairs(self.h, ctypes.c_float(R), ctypes.byref(t)), "radius_pairs")
        return t.value


def select_topk(idx, ratio, k):
    idx = np.ascontiguousarray(idx, np.int32)
    ratio = np.ascontiguousarray(ratio, np.float32)
    o = np.zeros(max(k, 1), np.int32)
    r = np.zeros(max(k, 1), np.float32)
    m = ctypes.c_int()
    rc = lib().bshot_select_topk(_ptr(idx), _ptr(ratio), len(idx), k, _ptr(o), _ptr(r), ctypes.byref(m))
    if rc < 0:
        raise BshotError("select_topk failed")
    return o[: m.value].copy(), r[: m.value].copy()


def ransac(src, tgt, cq, cm, max_iter=2000, thresh=1500.0):
    src = _f32(src).reshape(-1, 3)
    tgt = _f32(tgt).reshape(-1, 3)
    cq = np.ascontiguousarray(cq, np.int32)
    cm = np.ascontiguousarray(cm, np.int32)
    T = np.zeros(16, np.float32)
    iq = np.zeros(max(len(cq), 1), np.int32)
    im = np.zeros(max(len(cq), 1), np.int32)
    ni = ctypes.c_int()
    rc = lib().bshot_ransac(_ptr(src), len(src), _ptr(tgt), len(tgt), _ptr(cq), _ptr(cm), len(cq), max_iter,
                            ctypes.c_double(thresh), _ptr(T), _ptr(iq), _ptr(im), ctypes.byref(ni))
    if rc < 0:
        raise BshotError("ransac failed")
    return rc, T.reshape(4, 4), iq[: ni.value].copy(), im[: ni.value].copy()


def ransac_scores(cs, ct, hyp, thresh=1500.0, ctx=None):
    """Inlier counts of RANSAC hypotheses (3 correspondence positions each) over the pairs cs[i] ->
    ct[i]: on the GPU with a Context (csrc/ransac.hip k_ransac_score), on the host without."""
    cs = _f32(cs).reshape(-1, 3)
    ct = _f32(ct).reshape(-1, 3)
    hyp = np.ascontiguousarray(hyp, np.int32).reshape(-1, 3)
    cnt = np.zeros(max(len(hyp), 1), np.int32)
    h = ctx.h if ctx is not None else None
    rc = lib().bshot_ransac_scores(h, _ptr(cs), _ptr(ct), len(cs), _ptr(hyp), len(hyp), ctypes.c_double(thresh),
                                   _ptr(cnt))
    if rc < 0:
        raise BshotError("ransac_scores failed: %d" % rc)
    return cnt[: len(hyp)].copy()


class Odometry:
    """Headless odometry_test loop (bshot_odom)."""

    def __init__(self, device=0, params=None):
        self.L = lib()
        self.h = P()
        self.params = params if params is not None else default_params()
        rc = self.L.bshot_odom_create(ctypes.byref(self.h), device, ctypes.byref(self.params))
        if rc != 0:
            raise BshotError(f"bshot_odom_create failed ({rc})")

    def close(self):
        if self.h:
            self.L.bshot_odom_destroy(self.h)
            self.h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc < 0:
            raise BshotError(f"{what}: {self.L.bshot_odom_last_error(self.h).decode()} ({rc})", rc)
        return rc

    def process(self, xyz):
        xyz = _f32(xyz).reshape(-1, 3)
        st = FrameStats()
        self._chk(self.L.bshot_odom_process(self.h, _ptr(xyz), len(xyz), ctypes.byref(st)), "odom_process")
        return st

    def set_next_device(self, dptr, n):
        """Lookahead: the device cloud the next process_device call will receive."""
        self._chk(self.L.bshot_odom_set_next_device(self.h, P(dptr), n), "odom_set_next_device")

    def set_next2_device(self, dptr, n):
        """Lookahead depth 2: the device cloud of the process_device call after next."""
        self._chk(self.L.bshot_odom_set_next2_device(self.h, P(dptr), n), "odom_set_next2_device")

    def drain(self):
        """Wait for the lookahead work in flight (bshot_odom_drain); prefetched results stay ready."""
        self._chk(self.L.bshot_odom_drain(self.h), "odom_drain")

    def process_device(self, dptr, n):
        st = FrameStats()
        self._chk(self.L.bshot_odom_process_device(self.h, P(dptr), n, ctypes.byref(st)), "odom_process_device")
        return st

    def extract_device(self, dptr, n):
        """Frame-sharded mode: the extraction half of a device sweep as a float32 record
        (bshot_odom_extract_device); the set_next lookahead applies."""
        K = max(1, self.params.num_keypoints)
        cap = 8 + 15 * K + 3 * (n + 1) + 4 * min(n, K)  # k <= K, ISS points <= n, normals slots min(n, K)
        rec = np.zeros(cap, np.float32)
        ln = self._chk(self.L.bshot_odom_extract_device(self.h, P(dptr), n, _ptr(rec), cap), "odom_extract_device")
        return rec[:ln].copy()

    def process_record(self, rec):
        """Frame-sharded mode: the chain half of the next sweep from an extraction record. Raises
        BshotError with code ESTALE (and changes nothing) when the record was described over other
        stale normals than the sequence's: process that sweep with process[_device] instead."""
        rec = np.ascontiguousarray(rec, np.float32)
        st = FrameStats()
        self._chk(self.L.bshot_odom_process_record(self.h, _ptr(rec), len(rec), ctypes.byref(st)), "odom_process_record")
        return st

    def _get(self, fn, shape_cols, dtype, cap=1 << 20):
        buf = np.zeros((cap, shape_cols), dtype)
        n = fn(self.h, _ptr(buf), cap)
        if n < 0:
            return self._get(fn, shape_cols, dtype, -n)
        return buf[:n].copy()

    def keypoints(self):
        return self._get(self.L.bshot_odom_get_keypoints, 3, np.float32)

    def ratios(self):
        return self._get(self.L.bshot_odom_get_ratios, 1, np.float32)[:, 0]

    def bits(self):
        return self._get(self.L.bshot_odom_get_bits, 11, np.uint32)

    def iss(self):
        return self._get(self.L.bshot_odom_get_iss, 3, np.float32)

    def target(self, cap=1 << 20):
        xyz = np.zeros((cap, 3), np.float32)
        bits = np.zeros((cap, 11), np.uint32)
        n = self.L.bshot_odom_get_target(self.h, _ptr(xyz), _ptr(bits), cap)
        if n < 0:
            return self.target(-n)
        return xyz[:n].copy(), bits[:n].copy()

    def inliers(self, cap=1 << 16):
        q = np.zeros(cap, np.int32)
        m = np.zeros(cap, np.int32)
        n = self.L.bshot_odom_get_inliers(self.h, _ptr(q), _ptr(m), cap)
        if n < 0:
            return self.inliers(-n)
        return q[:n].copy(), m[:n].copy()

    def map_delta(self, cap=1 << 16):
        rec = np.zeros((cap, 15), np.float32)
        n = self.L.bshot_odom_map_delta(self.h, _ptr(rec), cap)
        if n < 0:
            return self.map_delta(-n)
        return rec[:n].copy()

    def replica_insert(self, replica, rec):
        rec = np.ascontiguousarray(rec, np.float32).reshape(-1, 15)
        self._chk(self.L.bshot_odom_replica_insert(self.h, replica, _ptr(rec), len(rec)), "replica_insert")

    def exchange(self, xchg, include_self=False):
        """Map offer of the last sweep -> every rank's GPU replicas over RCCL (bshot_odom_exchange)."""
        self._chk(self.L.bshot_odom_exchange(self.h, xchg.h, 1 if include_self else 0), "odom_exchange")

    def exchange_sim(self, xchg, peers):
        """bshot_odom_exchange_sim: the exchange plus `peers` simulated ranks' inserts (measurement)."""
        self._chk(self.L.bshot_odom_exchange_sim(self.h, xchg.h, int(peers)), "odom_exchange_sim")

    def gpu_replica_insert(self, replica, rec):
        rec = np.ascontiguousarray(rec, np.float32).reshape(-1, 15)
        self._chk(self.L.bshot_odom_gpu_replica_insert(self.h, replica, _ptr(rec), len(rec)), "gpu_replica_insert")

    def gpu_replica_size(self, replica):
        n = self.L.bshot_odom_gpu_replica_size(self.h, replica)
        if n < 0:
            raise BshotError(f"gpu_replica_size ({n})")
        return n

    def gpu_replica_query(self, replica, pos, rng=100000.0, cap=1 << 16):
        xyz = np.zeros((cap, 3), np.float32)
        bits = np.zeros((cap, 11), np.uint32)
        p = np.ascontiguousarray(pos, np.float32)
        n = self.L.bshot_odom_gpu_replica_query(self.h, replica, _ptr(p), ctypes.c_float(rng), _ptr(xyz), _ptr(bits),
                                                cap)
        if n < -1 and -n > cap:
            return self.gpu_replica_query(replica, pos, rng, -n)
        if n < 0:
            raise BshotError(f"gpu_replica_query ({n})")
        return xyz[:n].copy(), bits[:n].copy()

    def replica_size(self, replica):
        return self.L.bshot_odom_replica_size(self.h, replica)

    def context(self):
        return self.L.bshot_odom_ctx(self.h)

    def stage_times(self):
        ms = (ctypes.c_double * NSTAGES)()
        nl = (ctypes.c_int64 * NSTAGES)()
        self.L.bshot_stage_times(P(self.context()), ms, nl, NSTAGES)
        return {STAGE_NAMES[i]: (ms[i], nl[i]) for i in range(NSTAGES)}

    def set_option(self, name, value):
        if self.L.bshot_odom_set_option(self.h, name.encode(), int(value)) < 0:
            raise BshotError(f"set_option {name}")

    def upload(self, d_dst, h_src, n):
        """sweep upload (pinned host -> device) queued ahead of its lookahead work (bshot_odom_upload)"""
        self._chk(self.L.bshot_odom_upload(self.h, P(d_dst), P(h_src), int(n)), "upload")

    def set_metrics_file(self, path):
        """per-sweep JSON lines (counts, gate and its reasons, pose, host ms per phase); None stops"""
        self._chk(self.L.bshot_odom_set_metrics_file(self.h, (path or "").encode()), "set_metrics_file")

    def set_timing(self, on):
        self.L.bshot_set_timing(P(self.context()), 1 if on else 0)

    def stage_reset(self):
        self.L.bshot_stage_reset(P(self.context()))


class Exchange:
    """RCCL map exchange between ranks (bshot_xchg): id from rank 0 (unique_id), shared by the caller."""

    @staticmethod
    def unique_id():
        buf = (ctypes.c_char * 128)()
        if lib().bshot_xchg_unique_id(buf) != 0:
            raise BshotError("bshot_xchg_unique_id")
        return bytes(buf)

    def __init__(self, uid, nranks, rank, device, kmax):
        self.L = lib()
        self.h = P()
        buf = (ctypes.c_char * 128).from_buffer_copy(uid)
        rc = self.L.bshot_xchg_create(ctypes.byref(self.h), buf, nranks, rank, device, kmax)
        if rc != 0:
            raise BshotError(f"bshot_xchg_create ({rc})")

    def close(self):
        if self.h:
            self.L.bshot_xchg_destroy(self.h)
            self.h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KeypointMap:
    """Host keypoint map (myslam::Map) through the C ABI; no GPU needed."""

    def __init__(self):
        self.L = lib()
        self.h = P(self.L.bshot_map_create())

    def __del__(self):
        try:
            self.L.bshot_map_destroy(self.h)
        except Exception:
            pass

    def add(self, xyz, ratio, bits):
        xyz = np.ascontiguousarray(xyz, np.float32)
        bits = np.ascontiguousarray(bits, np.uint32)
        return self.L.bshot_map_add(self.h, _ptr(xyz), ctypes.c_float(ratio), _ptr(bits))

    def query(self, pos, rng=100000.0, cap=1 << 16):
        pos = np.ascontiguousarray(pos, np.float32)
        xyz = np.zeros((cap, 3), np.float32)
        bits = np.zeros((cap, 11), np.uint32)
        n = self.L.bshot_map_query(self.h, _ptr(pos), ctypes.c_float(rng), _ptr(xyz), _ptr(bits), cap)
        if n < 0:
            return self.query(pos, rng, -n)
        return xyz[:n].copy(), bits[:n].copy()

    def size(self):
        return self.L.bshot_map_size(self.h)

    def set_query_mode(self, mode):
        """0: visit the map's blocks when cheaper (default), 1: the reference's lookup loop."""
        if self.L.bshot_map_set_query_mode(self.h, int(mode)) < 0:
            raise BshotError("set_query_mode")

    @staticmethod
    def block_id(pos):
        pos = np.ascontiguousarray(pos, np.float32)
        return int(lib().bshot_map_block_id(_ptr(pos)))


# ---------------------------------------------------------------- synthetic input (not the product)
def pcap_load(path):
    """bshot_pcap_load: the 1206-B data packets of a pcap file and their capture times (reference rule)."""
    L = lib()
    n = ctypes.c_int()
    rc = L.bshot_pcap_load(str(path).encode(), None, None, 0, ctypes.byref(n))
    if rc < 0:
        raise BshotError(f"pcap_load {path} ({rc})")
    pk = np.zeros((max(n.value, 1), 1206), np.uint8)
    ut = np.zeros(max(n.value, 1), np.int64)
    rc = L.bshot_pcap_load(str(path).encode(), _ptr(pk), _ptr(ut), n.value, ctypes.byref(n))
    if rc < 0:
        raise BshotError(f"pcap_load {path} ({rc})")
    return pk[: n.value].copy(), ut[: n.value].copy()


def _synth_lib():
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} not built")
        _synth = ctypes.CDLL(SYNTH_PATH)
    return _synth


def synth_lasers(frame, sensor=2, seed=42, max_range=120000.0, sensor_height=2450.0):
    """One rotation of synthetic Velodyne laser records (tools/synth.cpp synth_lasers), firing order.
    sensor 0 HDL-64, 1 VLP-128 style, 2 HDL-32E."""
    cap = 300000
    buf = np.zeros(cap, LASER_DTYPE)
    n = _synth_lib().synth_lasers(sensor, seed, frame, ctypes.c_float(max_range), ctypes.c_float(sensor_height),
                                  _ptr(buf), cap)
    if n < 0:
        raise RuntimeError("synth capacity")
    return buf[:n].copy()


def synth_sweep(frame, sensor=0, seed=42, no_ground=False, max_range=120000.0):
    """Deterministic synthetic Velodyne sweep (b-shot-slam_amd/tools/synth.cpp), sensor frame, mm."""
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise RuntimeError(f"{SYNTH_PATH} not built")
        _synth = ctypes.CDLL(SYNTH_PATH)
    cap = 300000
    buf = np.zeros((cap, 3), np.float32)
    pose = np.zeros(16, np.float32)
    n = _synth.synth_sweep(sensor, seed, frame, 1 if no_ground else 0, ctypes.c_float(max_range), _ptr(buf), cap,
                           _ptr(pose))
    if n < 0:
        raise RuntimeError("synth capacity")
    return buf[:n].copy(), pose.reshape(4, 4)
