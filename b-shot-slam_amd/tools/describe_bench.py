"""Diagnostic: standalone (uncontended) describe timing per stage for describe2 knob settings.
usage: python describe_bench.py [knob values, default 2 1]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

# DESCRIBE_CFG=5: BASELINE config 5 (VLP-128 style sweep, K = 4096, SHOT radius 5000 mm)
cfg5 = os.environ.get("DESCRIBE_CFG") == "5"
pc, _ = bshot_py.synth_sweep(3, sensor=1 if cfg5 else 0)
c = bshot_py.Context(0, bshot_py.default_params(shot_radius=5000.0) if cfg5 else None)
c.set_cloud(pc)
idx, rat = c.seg_ratio()
kp, _ = bshot_py.select_topk(idx, rat, 4096 if cfg5 else 2048)
kps = pc[kp]
ref = None
# arguments: name=value option sets ("chunk_blocks=2048,dev_plan=0"); none: the defaults
for arg in sys.argv[1:] or ["default"]:
    opts = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in arg.split(",")) if "=" in arg else {}
    for kk, vv in opts.items():
        c.set_option(kk, vv)
    label = arg
    c.describe(kps)
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        bits, shot, rf = c.describe(kps)
    st = c.stage_times()
    c.set_timing(False)
    same = ref is None or np.array_equal(bits, ref)
    ref = bits if ref is None else ref
    ms = {k: round(v[0] / 10, 4) for k, v in st.items() if v[1]}
    print(json.dumps({"options": label, "identical_bits": bool(same), "bits_sha": hashlib.sha1(bits.tobytes()).hexdigest()[:12],
                      "shot_sha": hashlib.sha1(shot.tobytes()).hexdigest()[:12], "total_ms": round(sum(ms.values()), 4), **ms}))
c.close()
