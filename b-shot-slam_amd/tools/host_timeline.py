"""Median per-sweep timeline of both host threads from a BSHOT_HOST_TRACE csv (name, steady-clock ns):
every mark's offset from its sweep's M_frame (main thread) -- the worker's W_* marks belong to the
lookahead sweep it describes, so they are placed against the M_frame that precedes them.
usage: python host_timeline.py host.csv"""
import csv
import sys
from collections import defaultdict

rows = [(n, int(t)) for n, t in csv.reader(open(sys.argv[1]))]
rows.sort(key=lambda r: r[1])
frames = [t for n, t in rows if n == "M_frame"]
off = defaultdict(list)
fi = -1
seen = defaultdict(int)
for n, t in rows:
    while fi + 1 < len(frames) and frames[fi + 1] <= t:
        fi += 1
        seen = defaultdict(int)
    if fi < 1 or fi >= len(frames) - 1:
        continue
    k = f"{n}#{seen[n]}" if seen[n] else n
    seen[n] += 1
    off[k].append((t - frames[fi]) / 1e6)
per = sorted((b - a) / 1e6 for a, b in zip(frames, frames[1:]))
print(f"sweeps {len(per)}  period median {per[len(per) // 2]:.3f} ms  p10 {per[len(per) // 10]:.3f}  p90 {per[9 * len(per) // 10]:.3f}")
items = []
for k, v in off.items():
    if len(v) < len(per) // 2:
        continue
    v.sort()
    items.append((v[len(v) // 2], k, v[len(v) // 10], v[9 * len(v) // 10], len(v)))
for med, k, p10, p90, n in sorted(items):
    print(f"{med:8.3f}  {k:22s} p10 {p10:7.3f} p90 {p90:7.3f} n={n}")
