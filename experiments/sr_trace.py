"""Per-variant SR kernel durations from a rocprofv3 kernel-trace CSV of experiments/sr_variants.py."""
import csv, glob, sys
import numpy as np
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "seg_ratio" in r["Kernel_Name"] or "k_sr_tiles" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sr = [(r["Kernel_Name"].split("(")[0], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
main = [x for x in sr if "seg_ratio" in x[0]]
tiles = [x[1] for x in sr if "k_sr_tiles" in x[0]]
print("k_sr_tiles median us", np.median(tiles) if tiles else None)
for i in range(0, len(main), 15):
    d = [x[1] for x in main[i:i + 15]]
    print(i // 15, main[i][0], f"median {np.median(d):.1f} us min {min(d):.1f}")
