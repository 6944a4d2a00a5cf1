import sys, time, json
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bshot_py, numpy as np
c = bshot_py.Context(0)
pc, _ = bshot_py.synth_sweep(3)
c.set_cloud(pc)
c.seg_ratio()
s = c.knn_stats()
q = s[0]
print(json.dumps({"queries": q, "steps": s[1:5], "chunks_per_q": s[5]/q, "refine": s[7], "avgP": s[8]/q, "avg_need": s[9]/q, "avg_total": s[10]/q, "streamed": s[11]}))
