"""Diagnostic: standalone k_seg_ratio time (stage events, 10 launches) and kNN work counters per query
on one synthetic HDL-64 sweep, for the library BSHOT_LIB selects (A/B of builds).
usage: python sr_bench.py [option sets "name=value,name=value" ...]  (none: the defaults); the ratios
of every set must be bit-identical to the first's."""
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
    idx, rat = c.seg_ratio()
    cur = np.concatenate([idx.view(np.uint32), rat.view(np.uint32)])
    same = ref is None or np.array_equal(cur, ref)
    ref = cur if ref is None else ref
    c.set_timing(True)
    c.stage_reset()
    for _ in range(10):
        c.set_cloud(pc)
        c.seg_ratio()
    st = c.stage_times()
    c.set_timing(False)
    s = [int(x) for x in c.knn_stats()]
    q = max(1, s[0])
    print(json.dumps({"lib": os.environ.get("BSHOT_LIB", "tree"), "options": arg, "identical": bool(same),
                      "ms_per_launch": round(st["seg_ratio"][0] / 10, 4),
                      "chunks_per_q": round(s[5] / q, 3), "failed_chunks_per_q": round(s[26] / q, 3),
                      "streaming_path_frac": round(s[11] / q, 4), "in_radius_per_q": round(s[10] / q, 1),
                      "refine_passes_per_q": round(s[7] / q, 4),
                      # bounded passes (runs of cell-order queries): delivered / fell back to the ladder
                      "bounded_frac": round(s[27] / q, 4), "bounded_fallback_frac": round(s[28] / q, 4),
                      # per-query wave-clock shares (DIAG launch): ladder + streaming, selection from
                      # the LDS list, selection on the streaming path, the ratio (centroid + signs)
                      "cycle_share": {k: round(s[i] / max(1, s[12] + s[13] + s[14] + s[15]), 3)
                                      for k, i in (("ladder", 12), ("select", 13), ("select_stream", 14), ("ratio", 15))}}))
c.close()
