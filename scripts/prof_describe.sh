#!/bin/bash
# per-kernel times of the standalone describe (tools/describe_bench.py) under rocprofv3
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pd}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG -o t --output-format csv -- \
    python3 $R/b-shot-slam_amd/tools/describe_bench.py ${2:-2} > $R/gpurun_out/$TAG.log 2>&1 || exit $?
python3 - "$R/gpurun_out/$TAG/t_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:30]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
PY
