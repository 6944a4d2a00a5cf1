"""Per-kernel write bytes per dispatch from a rocprofv3 --pmc WRITE_SIZE pass (KiB -> bytes, as
scripts/prof_summary.py): usage wsize.py <counter_collection.csv> [kernel substrings...]"""
import collections
import csv
import sys

agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "WRITE_SIZE":
        agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]) * 1024.0)
keys = sys.argv[2:] or ["k_shot_gather_b", "k_shot_rank", "k_hist_fused", "k_lrf_chunks"]
for name, v in sorted(agg.items()):
    if any(k in name for k in keys):
        print(f"  {name[:48]:48s} n={len(v):4d} write {sum(v) / len(v) / 1e6:9.2f} MB/dispatch")
