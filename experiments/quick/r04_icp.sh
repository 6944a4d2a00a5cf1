#!/bin/bash
# round 4: ICP step/NN kernels -- ICP and whole-frame parity tests, then an A/B of bench lines
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
N=${1:-2}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "icp or odometry or sequence or edge or shard or golden or smoke or describe or rank" > $O/r04_icp_pytest.log 2>&1
rc=$?; tail -3 $O/r04_icp_pytest.log; [ $rc -eq 0 ] || exit $rc
bash experiments/quick/ab_multi.sh $N experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so ${@:2}
