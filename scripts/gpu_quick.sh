#!/bin/bash
# quick GPU check: selected tests (-k expression) then a bench line at the default and driver sizes
# usage (via gpurun): bash scripts/gpu_quick.sh "<pytest -k expr>" [tag] [extra bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
K=${1:-icp}
TAG=${2:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest_$TAG.log 2>&1
rc=$?; tail -3 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${@:3} > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json &&
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ${@:3} > $O/bench_driver_$TAG.json 2>> $O/bench_$TAG.err && cat $O/bench_driver_$TAG.json
