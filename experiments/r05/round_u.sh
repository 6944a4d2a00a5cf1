#!/bin/bash
# round 5 session u: ICP candidate-list capacity 64 / 256 (libbshot_lc64 / lc256) vs 128 (product):
# ICP / odometry GPU tests on each variant, alternating bench A/B/C with per-sweep ICP waits
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05u}
L=b-shot-slam_amd/lib
for V in lc64 lc256; do
  BSHOT_LIB=$R/$L/exp/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp or odom" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; tail -1 $O/${T}_pytest_$V.log; [ $rc -eq 0 ] || exit $rc
done
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/exp/libbshot_lc64.so $L/exp/libbshot_lc256.so | tee $O/${T}_ab_listcap.txt || exit 1
python experiments/r05/icp_waits.py $O/abm_libbshot_amd_*.err $O/abm_libbshot_lc64_*.err $O/abm_libbshot_lc256_*.err | tee $O/${T}_icp_waits.txt
