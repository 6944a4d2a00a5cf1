"""Diagnostic: run the config-3 sequence (K=600) through two option sets side by side and report
the first frame where anything differs (stats, targets, inliers, pose).
usage: python seq_bisect.py frames "optA" "optB"   (opts: name=value,name=value)"""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import bshot_py  # noqa: E402

F = int(sys.argv[1])
opts = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv) for a in sys.argv[2:4]]
ods = []
for o in opts:
    od = bshot_py.Odometry(0, bshot_py.default_params(num_keypoints=600))
    for k, v in o.items():
        od.set_option(k, v)
    ods.append(od)
fields = ["n_valid_ratios", "n_keypoints", "n_target", "n_mutual", "n_inliers", "icp_iters", "gated", "map_size"]
for f in range(F):
    xyz, _ = bshot_py.synth_sweep(f)
    st = [od.process(xyz) for od in ods]
    a = [[getattr(s, n) for n in fields] for s in st]
    ta = [od.target() for od in ods]
    same_t = np.array_equal(ta[0][0].view(np.uint32), ta[1][0].view(np.uint32)) and np.array_equal(ta[0][1], ta[1][1])
    inl = [od.inliers() for od in ods]
    same_i = all(np.array_equal(x, y) for x, y in zip(inl[0], inl[1]))
    pose = [np.array(s.pose, np.float32).view(np.uint32) for s in st]
    tr = [np.array(s.T_ransac, np.float32).view(np.uint32) for s in st]
    if a[0] != a[1] or not same_t or not same_i or not np.array_equal(pose[0], pose[1]) or not np.array_equal(tr[0], tr[1]):
        print("first difference at frame", f)
        print(dict(zip(fields, zip(a[0], a[1]))))
        print("targets identical:", same_t, "inliers identical:", same_i, "T_ransac identical:", np.array_equal(tr[0], tr[1]))
        if not same_t and len(ta[0][0]) == len(ta[1][0]):
            d = np.nonzero(np.any(ta[0][0] != ta[1][0], axis=1) | np.any(ta[0][1] != ta[1][1], axis=1))[0]
            print("target rows differing:", len(d), d[:10], ta[0][0][d[:3]], ta[1][0][d[:3]])
        break
    if f % 50 == 0:
        print("frame", f, "ok", a[0], flush=True)
else:
    print("no difference in", F, "frames")
