"""Diagnostic: step-by-step fine-ladder (4-grid) SR with progress prints (teardown/hang hunt)."""
import faulthandler
import os
import sys

faulthandler.dump_traceback_later(int(os.environ.get("HT_TIMEOUT", "40")), exit=True)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "b-shot-slam_amd"))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
c.set_option("ladder_grids", 4)
print("opt", flush=True)
c.set_cloud(pc)
c.sync()
print("cloud", flush=True)
idx, rat = c.seg_ratio()
print("sr", len(idx), flush=True)
c2 = bshot_py.Context(0)
c2.set_cloud(pc)
i2, r2 = c2.seg_ratio()
print("ref sr", np.array_equal(idx, i2) and np.array_equal(rat.view(np.uint32), r2.view(np.uint32)), flush=True)
c2.close()
c.close()
print("closed", flush=True)
