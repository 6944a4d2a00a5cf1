#!/bin/bash
# rank kernel with LDS bitonic spans: describe parity, standalone describe with each rank kernel,
# bench A/B of the rank choice at config 2 and config 5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "describe or golden or shot or config5 or rank" > $O/r04_rankwg_pytest.log 2>&1
rc=$?; tail -1 $O/r04_rankwg_pytest.log; [ $rc -eq 0 ] || { tail -30 $O/r04_rankwg_pytest.log; exit $rc; }
timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py rank_wg=0 rank_wg=1 || exit 1
bash experiments/quick/ab_opts.sh 2 rank_wg=0 rank_wg=1 || exit 1
bash experiments/quick/ab_opts.sh 1 rank_wg=0 rank_wg=1 -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10
