"""Per-sweep ICP tail vs the grid searches of the persistent iterations kernel (bench stderr written
under BENCH_INTERVALS=1): is the slow sweeps' wait for iterations 1.. explained by sources that left
their candidate lists (bshot_work_counters [9], per-sweep differences)?
usage: python experiments/r06/icp_tail.py <bench.err>..."""
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
    W = np.diff(np.array(d["work_per_sweep"], float), axis=0)
    rest = (W[:, 2] - W[:, 8]) / 1e6
    gs = W[:, 9]
    print(f"{f}: sweeps {len(iv)}; grid searches per sweep mean {gs.mean():.1f} median {np.median(gs):.0f} "
          f"p90 {np.percentile(gs, 90):.0f} max {gs.max():.0f}; corr(rest wait, grid searches) "
          f"{np.corrcoef(rest, gs)[0, 1]:+.2f}, corr(interval, grid searches) {np.corrcoef(iv, gs)[0, 1]:+.2f}")
    for lo, hi in ((0, 5), (5, 15), (15, 30), (30, 60), (60, 1e9)):
        m = (gs >= lo) & (gs < hi)
        if m.any():
            print(f"  grid searches [{lo}, {hi}): {m.sum():4d} sweeps, rest wait median {np.median(rest[m]):.3f} "
                  f"p90 {np.percentile(rest[m], 90):.3f} ms, interval median {np.median(iv[m]):.3f}")
