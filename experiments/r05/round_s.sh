#!/bin/bash
# round 5 session s: k_icp_iterations capped at 96 VGPRs (product, ICPH_WPE 5) vs uncapped
# (libbshot_fold = HEAD d0a9ad4): ICP / odometry GPU tests, alternating bench A/B with per-sweep ICP waits
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05s}
A=b-shot-slam_amd/lib/libbshot_amd.so; B=b-shot-slam_amd/lib/exp/libbshot_fold.so
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1
rc=$?; tail -2 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $A $B | tee $O/${T}_ab_icp_wpe.txt || exit 1
python experiments/r05/icp_waits.py $O/abm_libbshot_amd_*.err $O/abm_libbshot_fold_*.err | tee $O/${T}_icp_waits.txt
