#!/bin/bash
# round 6 session 6: ICP sources per iteration wave (ICPH_SRC 8/16/32 vs 64) -- ICP tests on each,
# alternating benches with per-sweep ICP tails; onesweep ladder sort variant
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06f}
L=b-shot-slam_amd/lib
for V in s16 s8 os; do
  BSHOT_LIB=$R/$L/ab/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp or odometry_hdl64 or seg_ratio_bit" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; echo "$V: $(tail -1 $O/${T}_pytest_$V.log)"; [ $rc -eq 0 ] || exit $rc
done
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_s16.so $L/ab/libbshot_s8.so $L/ab/libbshot_s32.so $L/ab/libbshot_os.so | tee $O/${T}_ab.txt || exit 1
for V in amd s16 s8 s32 os; do python experiments/r06/icp_tail.py $O/abm_libbshot_${V}_*.err; done > $O/${T}_icp_tail.txt
grep -h "grid searches per sweep\|\[60" $O/${T}_icp_tail.txt
