"""Condense one gpu_round.sh profile set into tracked files under profiles/.

    python scripts/prof_summary.py r01   # reads gpurun_out/{prof,pmc_fetch,pmc_write}_r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary, verbatim) and
profiles/<tag>_pmc.json: per kernel, mean FETCH_SIZE / WRITE_SIZE per dispatch in bytes.
FETCH_SIZE is reported by rocprofv3 in KiB and, on gfx950, counts 128-B requests at 64 B
(MI355X_MICROARCH.md "HBM"), so hbm_read_bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE is KiB as is.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main(tag):
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, f"prof_{tag}", "trace_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, bench.py --steps 5 ({tag})",
           "correction": "hbm_read_bytes = FETCH_SIZE[KiB] * 1024 * 2 (gfx950 half-count); "
                         "hbm_write_bytes = WRITE_SIZE[KiB] * 1024",
           "kernels": {}}
    for ctr, sub, scale in (("FETCH_SIZE", "fetch", 2048.0), ("WRITE_SIZE", "write", 1024.0)):
        rows = list(csv.DictReader(open(os.path.join(src, f"pmc_{sub}_{tag}", f"{sub}_counter_collection.csv"))))
        agg = collections.defaultdict(list)
        for r in rows:
            if r["Counter_Name"] == ctr:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            e = out["kernels"].setdefault(k, {"dispatches": len(v)})
            e["hbm_read_bytes" if sub == "fetch" else "hbm_write_bytes"] = sum(v) / len(v) * scale
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    # per-kernel median launch duration from the same kernel trace (the rocprofv3 mean is skewed by
    # the cold first launches and by the launch that overlaps process teardown)
    tr = os.path.join(src, f"prof_{tag}", "trace_kernel_trace.csv")
    if os.path.exists(tr):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        with open(os.path.join(dst, f"{tag}_kernel_median.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "launches", "median_us", "mean_us", "min_us", "max_us"])
            for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
                v.sort()
                w.writerow([k, len(v), f"{v[len(v) // 2]:.1f}", f"{sum(v) / len(v):.1f}", f"{v[0]:.1f}", f"{v[-1]:.1f}"])
    pre = os.path.join(src, f"prof_pre_{tag}", "t_kernel_stats.csv")
    if os.path.exists(pre):
        shutil.copy(pre, os.path.join(dst, f"{tag}_preprocess_kernel_stats.csv"))
    for f in (f"pre_bench_{tag}.json", f"prof_bench_{tag}.json", f"bench_{tag}.json", f"bench_{tag}.err", f"pytest_gpu_{tag}.log", f"smoke_{tag}.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f"{tag}_{f.replace('_' + tag, '')}"))
    print(json.dumps({k: v for k, v in out["kernels"].items() if "k_seg_ratio" in k or "k_shot_hist" in k}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
