#!/bin/bash
# kernel-level timing of the bench path: rocprofv3 --kernel-trace --stats, summary printed
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pq}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG -o t --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 $2 $3 $4 > $R/gpurun_out/$TAG.log 2>&1 || exit $?
python3 - "$R/gpurun_out/$TAG/t_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:24]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
PY
