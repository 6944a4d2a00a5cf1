"""Diagnostic: standalone k_seg_ratio time (stage events, 10 launches) and kNN work counters per query
on one synthetic HDL-64 sweep, for the library BSHOT_LIB selects (A/B of builds)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bshot_py  # noqa: E402

pc, _ = bshot_py.synth_sweep(3)
c = bshot_py.Context(0)
c.set_cloud(pc)
c.seg_ratio()
c.set_timing(True)
c.stage_reset()
for _ in range(10):
    c.set_cloud(pc)
    c.seg_ratio()
st = c.stage_times()
c.set_timing(False)
s = [int(x) for x in c.knn_stats()]
q = max(1, s[0])
print(json.dumps({"lib": os.environ.get("BSHOT_LIB", "tree"), "ms_per_launch": round(st["seg_ratio"][0] / 10, 4),
                  "chunks_per_q": round(s[5] / q, 3), "failed_chunks_per_q": round(s[26] / q, 3),
                  "streaming_path_frac": round(s[11] / q, 4), "in_radius_per_q": round(s[10] / q, 1),
                  "refine_passes_per_q": round(s[7] / q, 4)}))
c.close()
