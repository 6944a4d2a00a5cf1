"""Diagnostic: standalone ISS stage time (grid + lane kernel + overflow kernel + NMS, stage events, 10
launches) on one synthetic HDL-64 sweep, for the library BSHOT_LIB selects (A/B of builds).
usage: python iss_bench.py [option sets "name=value,..."]; every set's ISS indices must equal the first's."""
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
    out = c.iss()
    same = ref is None or np.array_equal(out, ref)
    ref = out.copy() if ref is None else ref
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        c.set_cloud(pc)
        c.iss()
    st = c.stage_times()
    c.set_timing(False)
    print(json.dumps({"lib": os.environ.get("BSHOT_LIB", "tree"), "options": arg, "identical": bool(same),
                      "n_iss": int(len(out)), **{k: round(v[0] / 10, 4) for k, v in st.items() if v[1]}}))
c.close()
