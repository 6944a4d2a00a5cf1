"""Diagnostic: ISS time per grid-cell setting (identical results required)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "b-shot-slam_amd"))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
ref = None
for cellm in (1, 2):
    c = bshot_py.Context(0)
    c.set_option("iss_cell", cellm)
    c.set_cloud(pc)
    c.iss()
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        c.set_cloud(pc)
        got = c.iss()
    st = c.stage_times()
    same = ref is None or np.array_equal(got, ref)
    ref = got if ref is None else ref
    print(json.dumps({"iss_cell": cellm, "iss_ms": st["iss"][0] / 10, "n_iss": len(got), "identical": bool(same)}),
          flush=True)
    c.close()
