"""Diagnostic: standalone k_seg_ratio time and kNN work counters per query for SR run lengths
(option sr_run: consecutive cell-order queries per wave). usage: python sr_run_ab.py [runs...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
c.set_cloud(pc)
ref = None
for run in [int(x) for x in sys.argv[1:]] or [1, 4, 8]:
    c.set_option("sr_run", run)
    idx, rat = c.seg_ratio()
    same = ref is None or (np.array_equal(idx, ref[0]) and np.array_equal(rat.view(np.uint32), ref[1].view(np.uint32)))
    ref = ref or (idx, rat)
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        c.set_cloud(pc)
        c.seg_ratio()
    st = c.stage_times()
    c.set_timing(False)
    s = [int(x) for x in c.knn_stats()]
    q = max(1, s[0])
    print(json.dumps({"run": run, "same_bits": bool(same), "ms_per_launch": round(st["seg_ratio"][0] / 10, 4),
                      "chunks_per_q": round(s[5] / q, 3), "failed_steps_per_q": round(s[25] / q, 3),
                      "failed_chunks_per_q": round(s[26] / q, 3), "skipped_steps_per_q": round(s[6] / q, 3),
                      "resolved_at_step": s[16:25]}))
c.close()
