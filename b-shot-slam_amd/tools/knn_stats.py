"""SR kNN work counters (bshot_debug_knn_stats): where k_seg_ratio's time goes per query.
kst: 0 queries, 5 chunks streamed, 6 steps skipped unstreamed, 7 refine passes, 8 bitonic P,
9 need, 10 in-radius total, 11 streaming-path queries, 12..15 cycles (ladder, fast select,
slow select, finish), 16+s queries resolved at ladder step s, 25 streamed ladder steps that fell short of max_nn, 26 their
chunks."""
import json
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import bshot_py  # noqa: E402

c = bshot_py.Context(0)
pc, _ = bshot_py.synth_sweep(3)
c.set_cloud(pc)
c.seg_ratio()
s = [int(x) for x in c.knn_stats()]
q = max(1, s[0])
cyc = s[12:16]
print(json.dumps({"queries": s[0], "chunks_per_q": s[5] / q, "skipped_steps_per_q": s[6] / q, "refine": s[7],
                  "avg_need": s[9] / q, "avg_total": s[10] / q, "streamed_path": s[11],
                  "cycles_per_q": {"ladder": cyc[0] / q, "fast_sel": cyc[1] / q, "slow_sel": cyc[2] / q,
                                   "finish": cyc[3] / q},
                  "resolved_at_step": s[16:16 + 9], "failed_steps_per_q": s[25] / q,
                  "failed_chunks_per_q": s[26] / q}))
