#!/bin/bash
# round 6 session 2: tests touched so far (corr stats, shard owner lookahead, ICP row, SR runs), then
# standalone SR per run length / grid ratio, then alternating bench lines over sr_run
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06b}
timeout -k 10 900 python -u -m pytest tests/test_odometry_gpu.py tests/test_shard_gpu.py tests/test_golden.py tests/test_parity_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "corr or shard or golden or icp or seg_ratio" > $O/${T}_pytest.log 2>&1
rc=$?; tail -3 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python b-shot-slam_amd/tools/sr_bench.py sr_run=1 sr_run=4 sr_run=8 sr_run=16 sr_run=32 sr_run=8,sr_bratio=200 sr_run=8,sr_bratio=400 > $O/${T}_sr_bench.txt 2>&1 || { cat $O/${T}_sr_bench.txt; exit 1; }
cat $O/${T}_sr_bench.txt
bash experiments/quick/ab_opts.sh 2 sr_run=1 sr_run=8 sr_run=16 | tee $O/${T}_ab_run.txt
