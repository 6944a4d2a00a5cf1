#!/bin/bash
# Fast iteration on the GPU box: stage parity + golden fixtures, then a bench line with stage ms.
# usage: bash scripts/gpu_quick.sh [tag] [extra pytest selection]
set -u
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q > $O/quick_pytest_$TAG.log 2>&1
rc=$?
tail -5 $O/quick_pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --profile-stages > $O/quick_bench_$TAG.json 2> $O/quick_bench_$TAG.err
rc=$?
cat $O/quick_bench_$TAG.json; tail -2 $O/quick_bench_$TAG.err
exit $rc
