#!/bin/bash
# round 6 session 1: the tests touched by the first commit (corr stats, shard owner lookahead, ICP row),
# then one bench line on HEAD
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06a}
timeout -k 10 600 python -u -m pytest tests/test_odometry_gpu.py tests/test_shard_gpu.py tests/test_golden.py tests/test_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "corr or shard or golden or icp" > $O/${T}_pytest.log 2>&1
rc=$?; tail -3 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cat $O/${T}_bench.json
