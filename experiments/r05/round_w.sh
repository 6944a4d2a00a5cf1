#!/bin/bash
# round 5 session w: ICP candidate-list capacity 256 / 512 (libbshot_lc256 / lc512, current sources) vs
# 128 (product): ICP / odometry GPU tests on each variant, alternating bench A/B/C at configs 1 and 5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05w}
L=b-shot-slam_amd/lib
for V in lc256 lc512; do
  BSHOT_LIB=$R/$L/exp/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp or odom" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; tail -1 $O/${T}_pytest_$V.log; [ $rc -eq 0 ] || exit $rc
done
rm -f $O/abm_*.err $O/abm_*.json
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/exp/libbshot_lc256.so $L/exp/libbshot_lc512.so | tee $O/${T}_ab_listcap.txt || exit 1
python experiments/r05/icp_waits.py $O/abm_libbshot_amd_*.err $O/abm_libbshot_lc256_*.err $O/abm_libbshot_lc512_*.err > $O/${T}_icp_waits.txt
bash experiments/quick/ab_multi.sh 1 $L/libbshot_amd.so $L/exp/libbshot_lc256.so $L/exp/libbshot_lc512.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_listcap_c5.txt
