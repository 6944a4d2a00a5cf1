#!/bin/bash
# per-kernel averages (rocprofv3 kernel trace) of a short bench run for each library: kstats_ab.sh <pattern> <lib>...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
PAT=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  T=$(basename $L .so)
  BSHOT_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ks_$T -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $R/gpurun_out/ks_$T.json 2>/dev/null || exit 1
  python3 - "$R/gpurun_out/ks_$T" "$PAT" "$T" <<'PY'
import csv, glob, sys, re
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if re.search(sys.argv[2], r["Name"]):
        print(sys.argv[3], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
  rm -rf $R/gpurun_out/ks_$T
done
