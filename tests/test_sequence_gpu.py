"""BASELINE config 3 over its full length: odometry_test's frame loop (test/odometry_test.cpp:122-346)
on 1000 synthetic HDL-64 sweeps, K=600, run through the product (bshot_odom, throughput mode with
the depth-2 lookahead the bench uses) and checked frame by frame against the committed golden
tests/golden/sequence_1000f.npz (made by tests/golden/make_sequence_1000f.py from the oracle; parity
unpinned vs PCL).

Per frame: every count of the chain (valid ratios, keypoints, ISS, targets M, mutual matches,
inliers, ICP iterations, gate, map size), the pose, T_ransac, h_diff and t_diff bits, and CRC32s of
the keypoints, the B-SHOT bits and the inlier pairs -- all bit-exact. This is the M ~ 10^4 matching
regime the short tests never reach. The end-point drift against the synthetic ground truth is
reported and written to gpurun_out/sequence_1000f_report.json when that
directory exists."""
import json
import os
import queue
import threading
import zlib

import numpy as np
import pytest

import bshot_py

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "sequence_1000f.npz")


def _crc(a):
    return zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF


def _bits(x):
    return np.ascontiguousarray(np.asarray(x, np.float32)).view(np.uint32)


def _producer(frames, q):
    for f in range(frames):
        q.put((f,) + bshot_py.synth_sweep(f))
    q.put(None)


@pytest.mark.timeout(600)
def test_config3_1000_frames_bit_exact():
    import torch

    g = np.load(GOLDEN)
    F, K = int(g["frames"]), int(g["k"])
    fields = [str(s) for s in g["stat_fields"]]
    q = queue.Queue(maxsize=8)
    threading.Thread(target=_producer, args=(F, q), daemon=True).start()
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=K))
    window = []  # (f, xyz, gt, device tensor) for f .. f+2
    retired = []
    poses = np.zeros((F, 16), np.float32)
    gts = np.zeros((F, 16), np.float32)
    try:
        done = False
        for f in range(F):
            while not done and len(window) < 3:
                item = q.get()
                if item is None:
                    done = True
                    break
                fi, xyz, gt = item
                assert _crc(xyz) == int(g["in_crc"][fi]), f"synthetic generator drift at frame {fi}"
                window.append((fi, xyz, gt, torch.from_numpy(xyz).to("cuda:0")))
            fi, xyz, gt, d = window[0]
            assert fi == f
            if len(window) > 1:
                od.set_next_device(window[1][3].data_ptr(), len(window[1][1]))
                if len(window) > 2:
                    od.set_next2_device(window[2][3].data_ptr(), len(window[2][1]))
            st = od.process_device(d.data_ptr(), len(xyz))
            got = [getattr(st, n) for n in fields]
            assert got == g["stats"][f].tolist(), (f, dict(zip(fields, zip(got, g["stats"][f].tolist()))))
            assert np.array_equal(_bits(st.pose), g["pose"][f].view(np.uint32)), f
            assert np.array_equal(_bits(st.T_ransac), g["T_ransac"][f].view(np.uint32)), f
            assert _bits([st.h_diff, st.t_diff]).tolist() == _bits([g["h_diff"][f], g["t_diff"][f]]).tolist(), f
            assert _crc(od.keypoints()) == int(g["kp_crc"][f]), f
            assert _crc(od.bits()) == int(g["bits_crc"][f]), f
            qi, mi = od.inliers()
            assert _crc(np.stack([qi, mi])) == int(g["inl_crc"][f]), f
            poses[f] = np.array(st.pose, np.float32)
            gts[f] = np.asarray(gt, np.float32).reshape(16)
            retired.append(window.pop(0))  # keep the last sweeps' device buffers alive a while
            del retired[:-4]
    finally:
        od.close()
    P, G = poses[-1].reshape(4, 4), gts[-1].reshape(4, 4)
    drift = float(np.linalg.norm(P[:3, 3].astype(np.float64) - G[:3, 3]))
    path = float(np.sum(np.linalg.norm(np.diff(gts[:, [3, 7, 11]].astype(np.float64), axis=0), axis=1)))
    yaw_err = float(np.arctan2(P[1, 0], P[0, 0]) - np.arctan2(G[1, 0], G[0, 0]))
    rep = {"frames": F, "keypoints": K, "end_point_drift_mm": drift, "path_length_mm": path,
           "drift_pct": 100.0 * drift / path, "end_yaw_error_rad": yaw_err,
           "final_M": int(g["stats"][-1][fields.index("n_target")]),
           "final_map_size": int(g["stats"][-1][fields.index("map_size")]),
           "gated_frames": int(g["stats"][:, fields.index("gated")].sum())}
    out = os.path.join(os.path.dirname(HERE), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "sequence_1000f_report.json"), "w") as fh:
            json.dump(rep, fh)
    print("config-3 1000-frame report:", rep)
