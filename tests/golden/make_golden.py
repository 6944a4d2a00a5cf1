"""Generate the committed golden fixtures (tests/golden/*.npz) from the oracle.

The reference cannot be built here (no PCL/Eigen/FLANN), so these vectors come from the CPU
restatement in oracle/ (parity unpinned vs PCL). They pin the restatement against
regressions and give the GPU path a fixed, reviewable target. Inputs are deterministic synthetic
sweeps (b-shot-slam_amd/tools/synth.cpp), subsampled to stay small.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "b-shot-slam_amd"), os.path.join(ROOT, "tests")]

import bshot_py  # noqa: E402  (synthetic input generator only)
import oracle_ref as orc  # noqa: E402

K = 64
STRIDE = 16


def stage_fixture():
    a = bshot_py.synth_sweep(0)[0][::STRIDE].copy()
    b = bshot_py.synth_sweep(1)[0][::STRIDE].copy()
    out = {"xyz_a": a, "xyz_b": b, "k": np.int32(K)}
    bits = []
    for tag, xyz in (("a", a), ("b", b)):
        sr_idx, sr_ratio = orc.seg_ratio(xyz)
        kp_idx, kp_ratio = orc.select_topk(sr_idx, sr_ratio, K)
        kps = xyz[kp_idx]
        nrm = orc.normals(xyz, kps)
        shot, rf = orc.shot(xyz, nrm, kps)
        bt = orc.binarize(shot)
        iss_idx, _ = orc.iss(xyz)
        out.update({f"sr_idx_{tag}": sr_idx, f"sr_ratio_{tag}": sr_ratio, f"kp_idx_{tag}": kp_idx,
                    f"normals_{tag}": nrm, f"shot_{tag}": shot, f"rf_{tag}": rf, f"bits_{tag}": bt,
                    f"iss_idx_{tag}": iss_idx})
        bits.append(bt)
    left, right, cq, cm = orc.match(bits[1], bits[0])
    out.update({"left": left, "right": right, "corr_q": cq, "corr_m": cm})
    np.savez_compressed(os.path.join(HERE, "stages_8k.npz"), **out)
    return out


def sequence_fixture(frames=3, stride=12, k=128):
    clouds = [bshot_py.synth_sweep(f)[0][::stride].copy() for f in range(frames)]
    od = orc.Odometry(orc.params(num_keypoints=k))
    out = {"k": np.int32(k)}
    for f, xyz in enumerate(clouds):
        st = od.process(xyz)
        q, m = od.inliers()
        out.update({f"xyz_{f}": xyz, f"pose_{f}": np.array(st.pose, np.float32).reshape(4, 4),
                    f"T_ransac_{f}": np.array(st.T_ransac, np.float32).reshape(4, 4),
                    f"kps_{f}": od.keypoints(), f"bits_{f}": od.bits(), f"inl_q_{f}": q, f"inl_m_{f}": m,
                    f"stats_{f}": np.array([st.n_valid_ratios, st.n_keypoints, st.n_iss, st.n_target, st.n_mutual,
                                            st.n_inliers, st.icp_iters, st.gated, st.map_size], np.int32)})
    np.savez_compressed(os.path.join(HERE, "sequence_3f.npz"), **out)
    return out


if __name__ == "__main__":
    s = stage_fixture()
    print("stages:", {k: getattr(v, "shape", v) for k, v in s.items()})
    q = sequence_fixture()
    print("sequence stats:", [q[f"stats_{f}"].tolist() for f in range(3)])
