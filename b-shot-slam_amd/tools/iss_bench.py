"""Diagnostic: standalone ISS stage time (stage events, 10 sweeps) on one synthetic HDL-64 sweep per
option set ("name=value,name=value"; none: the defaults); the ISS keypoints of every set must be
identical to the first's."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
ref = None
for arg in sys.argv[1:] or ["default"]:
    opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in arg.split(",")) if "=" in arg else {}
    for kk, vv in opts.items():
        c.set_option(kk, vv)
    c.set_cloud(pc)
    cur = c.iss()
    same = ref is None or np.array_equal(cur, ref)
    ref = cur if ref is None else ref
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        c.set_cloud(pc)
        c.iss()
    st = c.stage_times()
    c.set_timing(False)
    print(json.dumps({"lib": os.environ.get("BSHOT_LIB", "tree"), "options": arg, "identical": bool(same),
                      "iss_ms": round(st["iss"][0] / 10, 4), "grid_ms": round(st["grid"][0] / 10, 4),
                      "n_iss": int(len(cur))}))
c.close()
