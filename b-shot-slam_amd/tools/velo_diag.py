"""diagnostic: per-field mismatches of the GPU packet decode vs the oracle on random packets"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "b-shot-slam_amd"), os.path.join(R, "tests")]
import bshot_py  # noqa: E402
import oracle_ref as orc  # noqa: E402
from test_velodyne import random_packets  # noqa: E402

pk, ut = random_packets(132, 300)
ctx = bshot_py.Context(0)
rec, rs, rc = ctx.velodyne_decode(pk, ut, 32, 0)
orec, ocnt = orc.velodyne_decode(pk, ut, 32, 0)
for f in ("azimuth", "vertical", "distance", "intensity", "id", "time"):
    bad = np.nonzero(rec[f] != orec[f])[0]
    print(f, len(bad), bad[:5], rec[f][bad[:3]], orec[f][bad[:3]])
raw = rec.view(np.uint8).reshape(-1, 32) != orec.view(np.uint8).reshape(-1, 32)
print("bytes", raw.sum(axis=0))
ctx.close()
