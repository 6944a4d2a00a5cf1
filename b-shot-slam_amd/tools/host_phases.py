"""Median main-thread phase durations from a BSHOT_HOST_TRACE csv (name, steady-clock ns) of a bench
run without the profiler: gaps between consecutive main-thread marks of each sweep.
usage: python host_phases.py host.csv"""
import csv
import sys
from collections import defaultdict

rows = [(n, int(t)) for n, t in csv.reader(open(sys.argv[1]))]
main = [(n, t) for n, t in rows if n.startswith("M_")]
gaps = defaultdict(list)
for (a, ta), (b, tb) in zip(main, main[1:]):
    gaps[f"{a}->{b}"].append((tb - ta) / 1e6)
frames = [t for n, t in main if n == "M_frame"]
per = sorted((b - a) / 1e6 for a, b in zip(frames, frames[1:]))
print(f"sweeps {len(per)}  period median {per[len(per) // 2]:.3f} ms")
for k, v in sorted(gaps.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
    v.sort()
    if len(v) > len(per) // 2:
        print(f"{k:34s} n={len(v):4d} median {v[len(v) // 2]:.3f} ms  p90 {v[int(len(v) * 0.9)]:.3f}")
