#!/bin/bash
# standalone ICP: wall ms per call for the base and tree libraries, then a kernel trace of the tree's
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
for L in experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so; do
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/icp_bench.py 20 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r04_icpprof -o t --output-format csv -- python3 $R/b-shot-slam_amd/tools/icp_bench.py 10 > $O/r04_icpprof.log 2>&1 || exit 1
python3 - "$O/r04_icpprof/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['Percentage']):6.2f}%")
PY
