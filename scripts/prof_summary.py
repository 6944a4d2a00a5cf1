"""Condense one gpu_round.sh profile set into tracked files under profiles/.

    python scripts/prof_summary.py r01 [dst]   # reads gpurun_out/{prof,pmc_fetch,pmc_write}_r01
(dst: output directory, default profiles/; gpu_round.sh writes gpurun_out/summary_<tag> on the box so
that the raw traces can be dropped before gpurun copies gpurun_out/ back)

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


N_CU, N_SIMD = 256, 1024
DERIVED_DOC = {
    "time": "median launch duration of the kernel in the same round's kernel trace (prof_<tag>)",
    "cycles": "GRBM_GUI_ACTIVE / 8: rocprofv3 sums the counter over the 8 XCDs (GRBM / 8 / the PMC run's own "
              "dispatch duration = 2.4 GHz, checked on k_seg_ratio r02c)",
    "clock_ghz": "cycles / the PMC run's mean dispatch duration (Start/End timestamps of the counter CSV)",
    "valu_issue_frac": "SQ_INSTS_VALU x 2 cycles (wave64 fp32 issue on a 32-lane SIMD, MI355X_MICROARCH.md "
                       "per-instruction table) / (cycles x 1024 SIMDs): VALU issue share of the chip",
    "lds_busy_frac": "SQ_LDS_IDX_ACTIVE / (cycles x 256 CUs): LDS-array busy share",
    "lds_bank_conflict_frac": "SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE",
    "waves_per_cu": "SQ_WAVE_CYCLES x 4 (quad-cycles) / (cycles x 256 CUs): mean resident waves per CU",
    "wave_wait_frac": "SQ_WAIT_ANY / SQ_WAVE_CYCLES: waves parked on s_waitcnt / barriers",
    "wave_issue_stall_frac": "SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES: ready waves stalled at issue",
    "wave_active_frac": "SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES",
    "l2_hit_rate": "TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)",
    "limiter": "largest of valu_issue_frac / lds_busy_frac, or 'latency' when waves are parked most of their life "
               "(wave_wait_frac > 0.5) while both stay below 0.5",
}


def derive(e, c, dur, pmc_dur=None):
    g = lambda n: c.get(n)
    if dur:
        e["time_ms"] = round(dur * 1e3, 4)
    cyc = None
    if g("GRBM_GUI_ACTIVE"):
        cyc = g("GRBM_GUI_ACTIVE") / 8.0
        if pmc_dur:
            e["clock_ghz"] = round(cyc / pmc_dur / 1e9, 3)
    if cyc is None and dur:
        cyc = dur * 2.4e9
    if cyc:
        if g("SQ_INSTS_VALU") is not None:
            e["valu_issue_frac"] = round(g("SQ_INSTS_VALU") * 2.0 / (cyc * N_SIMD), 4)
        if g("SQ_LDS_IDX_ACTIVE") is not None:
            e["lds_busy_frac"] = round(g("SQ_LDS_IDX_ACTIVE") / (cyc * N_CU), 4)
        if g("SQ_WAVE_CYCLES") is not None:
            e["waves_per_cu"] = round(g("SQ_WAVE_CYCLES") * 4.0 / (cyc * N_CU), 2)
    if g("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_frac"] = round((g("SQ_LDS_BANK_CONFLICT") or 0.0) / g("SQ_LDS_IDX_ACTIVE"), 4)
    if g("SQ_WAVE_CYCLES"):
        for n, key in (("SQ_WAIT_ANY", "wave_wait_frac"), ("SQ_WAIT_INST_ANY", "wave_issue_stall_frac"),
                       ("SQ_ACTIVE_INST_ANY", "wave_active_frac")):
            if g(n) is not None:
                e[key] = round(g(n) / g("SQ_WAVE_CYCLES"), 4)
    if g("TCC_HIT_sum") is not None and (g("TCC_HIT_sum") + (g("TCC_MISS_sum") or 0)) > 0:
        e["l2_hit_rate"] = round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + (g("TCC_MISS_sum") or 0)), 4)
    v, l = e.get("valu_issue_frac", 0.0), e.get("lds_busy_frac", 0.0)
    if max(v, l) < 0.5 and e.get("wave_wait_frac", 0.0) > 0.5:
        e["limiter"] = "latency"
    elif v or l:
        e["limiter"] = "valu" if v >= l else "lds"


def main(tag, dst=None):
    src = os.path.join(ROOT, "gpurun_out")
    dst = dst or os.path.join(ROOT, "profiles")
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
    # SQ / TCC / TCP / GRBM passes (scripts/gpu_round.sh): per-dispatch means, then derived metrics
    raw = collections.defaultdict(lambda: collections.defaultdict(list))
    pdur = collections.defaultdict(list)
    for sub in ("sq1", "sq2", "tcc"):
        f = os.path.join(src, f"pmc_{sub}_{tag}", f"{sub}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            raw[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if sub == "tcc" and r["Counter_Name"] == "GRBM_GUI_ACTIVE" and "End_Timestamp" in r:
                pdur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    med = {}
    tr = os.path.join(src, f"prof_{tag}", "trace_kernel_trace.csv")
    if os.path.exists(tr):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
        med = {k: sorted(v)[len(v) // 2] for k, v in durs.items()}
    for k, ctrs in raw.items():
        e = out["kernels"].setdefault(k, {})
        c = {n: sum(v) / len(v) for n, v in ctrs.items()}
        e["counters"] = {n: round(v, 1) for n, v in c.items()}
        pd = pdur.get(k)
        derive(e, c, med.get(k), sum(pd) / len(pd) if pd else None)
    out["derived"] = DERIVED_DOC
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
    for f in (f"pre_bench_{tag}.json", f"prof_bench_{tag}.json", f"bench_{tag}.json", f"bench_driver_{tag}.json", f"host_phases_{tag}.txt", f"bench_{tag}.err", f"pytest_gpu_{tag}.log", f"smoke_{tag}.log"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f"{tag}_{f.replace('_' + tag, '')}"))
    print(json.dumps({k: v for k, v in out["kernels"].items() if "k_seg_ratio" in k}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01", sys.argv[2] if len(sys.argv) > 2 else None)
