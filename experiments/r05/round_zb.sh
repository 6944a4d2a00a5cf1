#!/bin/bash
# round 5 session zb: ICP list scan with 32 entries per round trip (libbshot_b32) and lists of 384 (libbshot_c384) vs 16 / 256 (product):
# ICP / odometry GPU tests on each variant, alternating bench A/B/C with per-sweep ICP waits
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05zb}
L=b-shot-slam_amd/lib
for V in b32 c384; do
  BSHOT_LIB=$R/$L/exp/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; tail -1 $O/${T}_pytest_$V.log; [ $rc -eq 0 ] || exit $rc
done
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/exp/libbshot_b32.so $L/exp/libbshot_c384.so | tee $O/${T}_ab_icp_batch.txt || exit 1
python experiments/r05/icp_waits.py $O/abm_libbshot_amd_*.err $O/abm_libbshot_b32_*.err $O/abm_libbshot_c384_*.err > $O/${T}_icp_waits.txt
