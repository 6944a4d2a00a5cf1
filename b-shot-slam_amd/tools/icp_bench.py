"""Diagnostic: standalone ICP (bshot_icp) on bench-sized inputs -- 2048 sources (a sweep's top-K
keypoints moved by a small rigid motion) against ~15k targets (keypoints of 8 sweeps) -- ms per call
(the host's wall time; the kernels of one call run back to back on the context's main stream)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bshot_py  # noqa: E402

c = bshot_py.Context(0)
tg = []
for f in range(8):
    pc, _ = bshot_py.synth_sweep(f)
    c.set_cloud(pc)
    idx, r = c.seg_ratio()
    k = np.argsort(-r, kind="stable")[:2048]
    tg.append(pc[idx[k]] + np.array([0, 800.0 * f, 0], np.float32))
tgt = np.concatenate(tg).astype(np.float32)
cs, sn = np.cos(0.01), np.sin(0.01)
src = (tg[3] @ np.array([[cs, -sn, 0], [sn, cs, 0], [0, 0, 1]], np.float32).T + np.array([300, -200, 50], np.float32))
src = src.astype(np.float32)
for _ in range(3):
    c.icp(src, tgt)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
t0 = time.perf_counter()
for _ in range(n):
    T, it = c.icp(src, tgt)
ms = (time.perf_counter() - t0) / n * 1e3
print(json.dumps({"ms_per_icp": round(ms, 4), "iters": it, "ns": len(src), "nt": len(tgt)}))
c.close()
