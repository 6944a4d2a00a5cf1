#!/bin/bash
# SR instruction mix per library (standalone sr_bench under rocprofv3 --pmc, one counter set per pass)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  T=$(basename $L .so)
  BSHOT_LIB=$R/$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD \
      -d $O/pmc_sr_$T -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/sr_bench.py > $O/pmc_sr_$T.log 2>&1 || { tail -5 $O/pmc_sr_$T.log; exit 1; }
  python3 - <<PY
import csv, glob, collections
f = glob.glob("$O/pmc_sr_$T/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'k_seg_ratio<false>' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print("$T", {k: round(sum(v) / len(v) / 130004, 1) for k, v in sorted(acc.items())}, "per query (mean over", len(acc['SQ_WAVES']), "launches)")
PY
done
