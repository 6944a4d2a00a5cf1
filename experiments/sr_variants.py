"""Diagnostic: SR kernel time and kNN work counters per tuning-knob setting (same results required)."""
import faulthandler
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "b-shot-slam_amd"))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

faulthandler.dump_traceback_later(int(os.environ.get("HT_TIMEOUT", "100")), exit=True)
pc, _ = bshot_py.synth_sweep(3)
ref = None
# each argument: comma-separated name=value context options, e.g. "ladder_grids=4,sr_start=50"
variants = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in v.split(",") if kv) for v in sys.argv[1:]] or [{}]
for opts in variants:
    if True:
        c = bshot_py.Context(0)
        for k, v in opts.items():
            c.set_option(k, v)
        c.set_cloud(pc)
        c.seg_ratio()
        c.set_timing(True)
        c.stage_reset()
        for _ in range(10):
            c.set_cloud(pc)
            idx, rat = c.seg_ratio()
        st = c.stage_times()
        c.set_timing(False)
        s = c.knn_stats()
        q = s[0]
        same = ref is None or (np.array_equal(idx, ref[0]) and np.array_equal(rat.view(np.uint32), ref[1].view(np.uint32)))
        if ref is None:
            ref = (idx, rat)
        print(json.dumps({"opts": opts, "sr_ms": st["seg_ratio"][0] / 10, "grid_ms": st["grid"][0] / 10,
                          "steps": s[16:25], "chunks_per_q": s[5] / q, "avg_total": s[10] / q, "streamed": s[11],
                          "refine": s[7], "skipped": s[6], "identical": bool(same),
                          "cyc_ladder": s[12] / q, "cyc_fastsel": s[13] / q, "cyc_streamsel": s[14] / q,
                          "cyc_math": s[15] / q,
                          "failed_steps_per_q": s[25] / q, "failed_chunks_per_q": s[26] / q}))
        c.close()
