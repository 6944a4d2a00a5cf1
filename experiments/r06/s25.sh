#!/bin/bash
# round 6 session 25: k_hist_fused with 5-wave workgroups at <= 96 VGPRs (nw5w5: 4 workgroups,
# 16 producers per CU) vs the product's 8 waves (2 workgroups, 14 producers), 10 waves at 96 and 5
# waves at 104 VGPRs; config 5 parity + benches for nw5w5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06z}
L=b-shot-slam_amd/lib
for V in nw10w5 nw5; do
  BSHOT_LIB=$R/$L/ab/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "describe_parity" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; echo "$V: $(tail -1 $O/${T}_pytest_$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for V in libbshot_amd ab/libbshot_nw5w5 ab/libbshot_nw10w5 ab/libbshot_nw5 libbshot_amd ab/libbshot_nw5w5 ab/libbshot_nw10w5 ab/libbshot_nw5; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_nw5w5.so | tee $O/${T}_ab.txt || exit 1
bash experiments/quick/ab_multi.sh 3 $L/ab/libbshot_nw5w5.so $L/libbshot_amd.so | tee $O/${T}_ab_rev.txt || exit 1
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_nw5w5.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_c5.txt || exit 1
