"""Config-3 divergence diagnostics (VERDICT r02 "Next round" #2), CPU only, on the oracle.

The committed 1000-frame config-3 golden (tests/golden/sequence_1000f.npz) is a diverging
trajectory: 35 % end-point drift, 840 of 1000 frames gated, median 7 RANSAC inliers. The GPU path
replays it bit for bit, so the question is whether that is the reference algorithm's behaviour on
this synthetic scene or a defect shared by the oracle and the kernels. Three diagnostics separate
the candidate causes:

  (i)   matching quality under ground-truth poses: the sequence is replayed with every frame's pose
        (and so the map and the reference keypoints) forced to the synthetic ground truth
        (pose override in the diagnostic oracle build), and each frame's mutual matches are scored
        against the ground truth (target within 300 mm / 1500 mm of GT * source keypoint);
  (ii)  the same with the normals-index bug of include/bshot_bits.h:59-86 corrected (every surface
        point gets its own normal; the reference writes keypoint k's normal into surface slot k and
        leaves the other slots zero, so SHOT's cosine coordinate is 5.0 for almost every neighbour);
  (iii) the same on an aperiodic scene variant (pole spacing 6-18 m instead of 12 m, hashed window
        layout instead of a 4 m period; tools/synth.cpp, scene seed bit 31).

Each is also run free (the odometry's own poses) for the drift it produces. Everything runs through
oracle/build/diag/liboracle_diag.so (make -C oracle diag), the restatement with two diagnostic-only
hooks compiled in; the parity oracle and the product never carry them.

    python tests/diag/config3_diag.py --frames 200 --out profiles/r03_config3_diag.json

TEST INFRASTRUCTURE ONLY (tests/ may load the oracle; nothing here is on the product path).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "b-shot-slam_amd"), os.path.join(ROOT, "tests")]
DIAG_LIB = os.path.join(ROOT, "oracle", "build", "diag", "liboracle_diag.so")
if not os.path.exists(DIAG_LIB):
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "diag"])
os.environ["ORACLE_LIB"] = DIAG_LIB  # oracle_ref loads the diagnostic build

import bshot_py  # noqa: E402  (synthetic input generator only)
import oracle_ref as orc  # noqa: E402

APERIODIC = 1 << 31


def mutual(od):
    L = orc.lib()
    cap = 1 << 16
    q = np.zeros(cap, np.int32)
    m = np.zeros(cap, np.int32)
    n = L.oracle_diag_get_mutual(od.h, q.ctypes.data_as(orc.P), m.ctypes.data_as(orc.P), cap)
    return q[:n].copy(), m[:n].copy()


def xf(T, p):
    return p @ T[:3, :3].T + T[:3, 3]


def rel_err(Ta, Tb):
    """translation (mm) and rotation (deg) of Ta^-1 Tb"""
    D = np.linalg.inv(Ta.astype(np.float64)) @ Tb.astype(np.float64)
    c = np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1)
    return float(np.linalg.norm(D[:3, 3])), float(np.degrees(np.arccos(c)))


def gt_pose(frame):
    """tools/synth.cpp's sensor pose at frame t (both synth_sweep and synth_lasers): yaw 0.5 deg *
    sin(2 pi t / 200), position (0, 800 t, 0); float32 like synth_sweep's pose_out"""
    yaw = 0.5 * np.pi / 180.0 * np.sin(2 * np.pi * frame / 200.0)
    c, s = np.cos(yaw), np.sin(yaw)
    P = np.array([[c, -s, 0, 0], [s, c, 0, 800.0 * frame], [0, 0, 1, 0], [0, 0, 0, 1]], np.float32)
    return P.astype(np.float64)


def laser_sweep(frame, sensor, seed):
    """odometry_test's input chain on synthetic laser returns: one rotation of the sensor
    (synth_lasers) through the oracle Preprocessor (test/odometry_test.cpp:32-33: vertical initial
    -0.6 rad, low-point threshold -1950 mm)."""
    L = bshot_py.synth_lasers(frame, sensor=sensor, seed=seed)
    xyz, _ = orc.preprocess(L, bshot_py.sensor_vertical_angles(sensor), -0.6, -1950.0)
    return xyz


def run(frames, fix_normals, aperiodic, gt_override, k, threads, run_icp=1, lasers=-1):
    od = orc.Odometry(orc.params(num_keypoints=k, run_icp=run_icp))
    orc.lib().oracle_diag_fix_normals(od.h, int(fix_normals))
    seed = 42 | (APERIODIC if aperiodic else 0)
    rows = []
    prev_kw = None
    prev_gt = None
    prev_pose = None
    t0 = time.time()
    for f in range(frames):
        if lasers >= 0:
            xyz, gt = laser_sweep(f, lasers, seed), gt_pose(f)
        else:
            xyz, gt = bshot_py.synth_sweep(f, seed=seed)
            gt = np.asarray(gt, np.float64).reshape(4, 4)
        if gt_override:
            G = np.ascontiguousarray(gt.astype(np.float32).reshape(16))
            orc.lib().oracle_diag_pose_override(od.h, G.ctypes.data_as(orc.P))
        st = od.process(xyz)
        kps = od.keypoints().astype(np.float64)
        tgt, _ = od.target()
        q, m = mutual(od)
        iq, im = od.inliers()
        kw = xf(gt, kps)  # GT world positions of this frame's keypoints
        row = {"frame": f, "n_mutual": st.n_mutual, "n_inliers": st.n_inliers, "gated": st.gated,
               "n_target": st.n_target, "map_size": st.map_size, "icp_iters": st.icp_iters}
        if f > 0 and len(q):
            d = np.linalg.norm(kw[q] - tgt[m].astype(np.float64), axis=1)
            row["mutual_gt_300"] = int((d < 300).sum())
            row["mutual_gt_1500"] = int((d < 1500).sum())
            di = np.linalg.norm(kw[iq] - tgt[im].astype(np.float64), axis=1) if len(iq) else np.zeros(0)
            row["inliers_gt_1500"] = int((di < 1500).sum())
        if prev_kw is not None and len(prev_kw):
            dd = np.sqrt(((kw[:, None, :] - prev_kw[None, :, :]) ** 2).sum(-1)).min(1)
            row["repeat_100"] = float((dd < 100).mean())
            row["repeat_300"] = float((dd < 300).mean())
        Tr = np.array(st.T_ransac, np.float64).reshape(4, 4)
        P = np.array(st.pose, np.float64).reshape(4, 4)
        if f > 0:
            # RANSAC's and the frame's own estimate of the motion since the previous frame, against GT
            ref_pose = prev_gt if gt_override else prev_pose
            if gt_override:  # RANSAC's absolute pose against GT (the map and reference are GT-placed)
                row["ransac_err_mm"], row["ransac_err_deg"] = rel_err(gt, Tr)
            step_est = np.linalg.inv(ref_pose) @ P
            step_gt = np.linalg.inv(prev_gt) @ gt
            row["step_est_mm"] = float(np.linalg.norm(step_est[:3, 3]))
            row["step_gt_mm"] = float(np.linalg.norm(step_gt[:3, 3]))
            row["step_err_mm"], row["step_err_deg"] = rel_err(step_gt, step_est)
        row["pose_err_mm"] = float(np.linalg.norm(P[:3, 3] - gt[:3, 3]))
        rows.append(row)
        prev_kw, prev_gt, prev_pose = kw, gt, (gt if gt_override else P)
        if f % 25 == 0:
            print(f"  frame {f}: mut={st.n_mutual} inl={st.n_inliers} gated={st.gated} "
                  f"gt300={row.get('mutual_gt_300')} rep100={row.get('repeat_100')} t={time.time() - t0:.0f}s",
                  flush=True)
    return rows


def summary(rows):
    r = rows[1:]

    def med(key):
        v = [x[key] for x in r if key in x]
        return float(np.median(v)) if v else None

    def mean(key):
        v = [x[key] for x in r if key in x]
        return float(np.mean(v)) if v else None

    last = rows[-1]
    return {
        "frames": len(rows),
        "mutual_median": med("n_mutual"), "mutual_gt_300_median": med("mutual_gt_300"),
        "mutual_gt_1500_median": med("mutual_gt_1500"), "mutual_gt_300_frac_mean":
            float(np.mean([x["mutual_gt_300"] / max(1, x["n_mutual"]) for x in r if "mutual_gt_300" in x])),
        "inliers_median": med("n_inliers"), "inliers_p90": float(np.percentile([x["n_inliers"] for x in r], 90)),
        "inliers_gt_1500_median": med("inliers_gt_1500"),
        "gated_frames": int(sum(x["gated"] for x in r)),
        "repeat_100_mean": mean("repeat_100"), "repeat_300_mean": mean("repeat_300"),
        "ransac_err_mm_median": med("ransac_err_mm"), "step_err_mm_median": med("step_err_mm"),
        "step_est_mm_median": med("step_est_mm"), "step_gt_mm_median": med("step_gt_mm"),
        "end_pose_err_mm": last["pose_err_mm"],
        "path_mm": 800.0 * (len(rows) - 1),
        "drift_pct": 100.0 * last["pose_err_mm"] / max(1.0, 800.0 * (len(rows) - 1)),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--keypoints", type=int, default=600)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--cases", default="ref_gt,fixn_gt,aper_gt,ref_free,fixn_free,aper_free,fixn_aper_free")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_config3_diag.json"))
    ap.add_argument("--lasers", type=int, default=-1,
                    help="sensor of synth_lasers (2: HDL-32E, the reference's own) fed through the oracle "
                         "Preprocessor, as odometry_test does; default: synth_sweep's HDL-64 point clouds")
    a = ap.parse_args()
    orc.set_point_threads(a.threads)
    orc.set_threads(a.threads)
    defs = {
        "ref_gt": (False, False, True), "fixn_gt": (True, False, True), "aper_gt": (False, True, True),
        "fixn_aper_gt": (True, True, True),
        "ref_free": (False, False, False), "fixn_free": (True, False, False), "aper_free": (False, True, False),
        "fixn_aper_free": (True, True, False),
        # (iv) the pose from RANSAC alone (setRunICP(false), test/odometry_test.cpp:41): is the
        # per-frame under-estimate of the motion the keypoint ICP's?
        "ref_noicp_free": (False, False, False, 0), "fixn_noicp_free": (True, False, False, 0),
    }
    out = {"frames": a.frames, "keypoints": a.keypoints, "lasers": a.lasers, "cases": {}}
    if os.path.exists(a.out):
        out = json.load(open(a.out))
    for c in a.cases.split(","):
        fixn, aper, gto = defs[c][:3]
        icp = defs[c][3] if len(defs[c]) > 3 else 1
        print(f"case {c}: fix_normals={fixn} aperiodic={aper} gt_override={gto} run_icp={icp}", flush=True)
        rows = run(a.frames, fixn, aper, gto, a.keypoints, a.threads, icp, a.lasers)
        out["cases"][c] = {"fix_normals": fixn, "aperiodic": aper, "gt_override": gto, "run_icp": icp,
                           "summary": summary(rows), "per_frame": rows}
        print(json.dumps({c: out["cases"][c]["summary"]}), flush=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
