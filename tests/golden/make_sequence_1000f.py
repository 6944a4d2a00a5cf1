"""Generate tests/golden/sequence_1000f.npz: BASELINE config 3 (odometry_test's frame loop,
test/odometry_test.cpp:122-346) over 1000 synthetic HDL-64 sweeps, K=600, run by the oracle.

The reference cannot be built here (no PCL/Eigen/FLANN), so the expected values come
from the CPU restatement in oracle/ (parity unpinned vs PCL). Per frame the fixture keeps what the
chain decides -- pose and T_ransac bits, the counts (valid ratios, keypoints, ISS, targets, mutual
matches, inliers, ICP iterations, gate, map size) -- plus CRC32s of the keypoints, the B-SHOT bits
and the inlier pairs, and a CRC32 of the input sweep so a change of the synthetic generator is
caught instead of read as a parity failure. The synthetic ground-truth pose is stored for the
end-point drift report.

    python tests/golden/make_sequence_1000f.py [--frames 1000] [--threads 8]

The oracle's per-point SR/ISS loops run on --threads threads (results do not depend on it).
"""
import argparse
import os
import sys
import time
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "b-shot-slam_amd"), os.path.join(ROOT, "tests")]

import bshot_py  # noqa: E402  (synthetic input generator only)
import oracle_ref as orc  # noqa: E402

STAT_FIELDS = ("n_points", "n_valid_ratios", "n_keypoints", "n_iss", "n_target", "n_mutual", "n_inliers",
               "icp_iters", "gated", "map_size")


def crc(a):
    return np.uint32(zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--keypoints", type=int, default=600)
    ap.add_argument("--out", default=os.path.join(HERE, "sequence_1000f.npz"))
    a = ap.parse_args()
    orc.set_point_threads(a.threads)
    orc.set_threads(a.threads)
    od = orc.Odometry(orc.params(num_keypoints=a.keypoints))
    F = a.frames
    out = {
        "frames": np.int32(F), "k": np.int32(a.keypoints), "scene_seed": np.int32(42), "sensor": np.int32(0),
        "stat_fields": np.array(STAT_FIELDS),
        "in_crc": np.zeros(F, np.uint32), "stats": np.zeros((F, len(STAT_FIELDS)), np.int32),
        "pose": np.zeros((F, 16), np.float32), "T_ransac": np.zeros((F, 16), np.float32),
        "h_diff": np.zeros(F, np.float32), "t_diff": np.zeros(F, np.float32),
        "kp_crc": np.zeros(F, np.uint32), "bits_crc": np.zeros(F, np.uint32), "inl_crc": np.zeros(F, np.uint32),
        "gt_pose": np.zeros((F, 16), np.float32),
    }
    t0 = time.time()
    for f in range(F):
        xyz, gt = bshot_py.synth_sweep(f)
        st = od.process(xyz)
        q, m = od.inliers()
        out["in_crc"][f] = crc(xyz)
        out["stats"][f] = [getattr(st, n) for n in STAT_FIELDS]
        out["pose"][f] = np.array(st.pose, np.float32)
        out["T_ransac"][f] = np.array(st.T_ransac, np.float32)
        out["h_diff"][f] = st.h_diff
        out["t_diff"][f] = st.t_diff
        out["kp_crc"][f] = crc(od.keypoints())
        out["bits_crc"][f] = crc(od.bits())
        out["inl_crc"][f] = crc(np.stack([q, m]))
        out["gt_pose"][f] = np.asarray(gt, np.float32).reshape(16)
        if f % 25 == 0 or f == F - 1:
            print(f"frame {f}: n={st.n_points} M={st.n_target} inl={st.n_inliers} gated={st.gated} "
                  f"map={st.map_size} t={time.time() - t0:.0f}s", flush=True)
    np.savez_compressed(a.out, **out)
    P, G = out["pose"][-1].reshape(4, 4), out["gt_pose"][-1].reshape(4, 4)
    print("end-point drift mm:", float(np.linalg.norm(P[:3, 3] - G[:3, 3])), "over",
          float(np.linalg.norm(G[:3, 3] - out["gt_pose"][0].reshape(4, 4)[:3, 3])), "mm")


if __name__ == "__main__":
    main()
