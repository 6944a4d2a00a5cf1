#!/bin/bash
# host timeline (both threads) of a bench run without the profiler, for each lib given
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
for L in "$@"; do
  T=$(basename $L .so)
  BSHOT_LIB=$R/$L BSHOT_HOST_TRACE=$O/host_$T.csv timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg --steps 100 --warmup 10 > $O/bench_host_$T.json 2>&1 || exit 1
  echo "== $T $(grep -o '"value": [0-9.]*' $O/bench_host_$T.json)"
  python b-shot-slam_amd/tools/host_timeline.py $O/host_$T.csv
done
