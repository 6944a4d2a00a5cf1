"""Per-sweep ICP wait split from a bench stderr file written under BENCH_INTERVALS=1.

usage: python experiments/r05/icp_waits.py <bench.err>...
Prints, per file, the ICP host phase and its waits (iteration 0 = the lists kernel, the rest = the
persistent iterations kernel) at several percentiles, and their correlation with the sweep interval.
"""
import json
import sys

import numpy as np

for f in sys.argv[1:]:
    d = None
    for line in open(f):
        if line.startswith('{"sweep_intervals_ms"'):
            d = json.loads(line)
    if d is None or not d.get("work_per_sweep"):
        print(f, "no per-sweep data")
        continue
    iv = np.array(d["sweep_intervals_ms"])[1:]
    P = np.array(d["per_sweep"], float)[1:]
    W = np.diff(np.array(d["work_per_sweep"], float), axis=0)
    icp, w_all, w0, step = P[:, 10], W[:, 2] / 1e6, W[:, 8] / 1e6, W[:, 4] / 1e6
    print(f"{f}: interval mean {iv.mean():.3f} median {np.median(iv):.3f} ms; ICP mean {icp.mean():.3f} "
          f"(waits: iteration 0 {w0.mean():.3f}, rest {(w_all - w0).mean():.3f}; host steps {step.mean():.3f})")
    for q in (50, 75, 90, 99):
        print(f"  p{q}: interval {np.percentile(iv, q):.3f} icp {np.percentile(icp, q):.3f} wait0 "
              f"{np.percentile(w0, q):.3f} rest {np.percentile(w_all - w0, q):.3f}")
    print(f"  corr(interval, icp) {np.corrcoef(iv, icp)[0, 1]:+.2f}  corr(interval, rest) "
          f"{np.corrcoef(iv, w_all - w0)[0, 1]:+.2f}")
