#!/bin/bash
# round 6 session 12: ICP kernels' LDS vs SR's leftover (5.8 KB per CU): lists kernel with 1-wave
# workgroups (2.6 KB) and iteration workgroups of 1 / 2 / 4 waves; product (lists 4, iterations 4)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06l}
L=b-shot-slam_amd/lib
BSHOT_LIB=$R/$L/ab/libbshot_l1w2.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp" > $O/${T}_pytest_l1w2.log 2>&1
rc=$?; echo "l1w2: $(tail -1 $O/${T}_pytest_l1w2.log)"; [ $rc -eq 0 ] || exit $rc
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_l1w1.so $L/ab/libbshot_l1w2.so $L/ab/libbshot_l1w4.so $L/ab/libbshot_l4w1.so $L/ab/libbshot_r5.so | tee $O/${T}_ab.txt || exit 1
for V in amd l1w1 l1w2 l1w4 l4w1 r5; do python experiments/r05/icp_waits.py $O/abm_libbshot_${V}_*.err | grep -v "p75\|p99\|corr"; done | tee $O/${T}_icp_waits.txt
