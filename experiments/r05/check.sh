#!/bin/bash
# round 5: selected GPU tests (-k expression), standalone SR counters, one bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
K=${1:-shard}
TAG=${2:-r05}
echo "[check] $(date +%T) pytest -k $K"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest_$TAG.log 2>&1
rc=$?; tail -5 $O/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "[check] $(date +%T) sr_bench"
timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py > $O/sr_$TAG.json 2>&1 && cat $O/sr_$TAG.json || exit 1
echo "[check] $(date +%T) bench"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-upload-leg > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json
