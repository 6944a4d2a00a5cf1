#!/bin/bash
# round 6 session 24: k_hist_fused workgroup shapes: product (8 waves, 104 VGPRs: 2 workgroups per CU)
# vs 6 waves at <= 80 VGPRs (spills), 5 and 4 waves at <= 96, 16 waves: describe parity per
# variant, standalone describe, alternating benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06y}
L=b-shot-slam_amd/lib
for V in nw6w6 nw5w5 nw4w5 nw16; do
  BSHOT_LIB=$R/$L/ab/libbshot_$V.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "describe_parity or config5" > $O/${T}_pytest_$V.log 2>&1
  rc=$?; echo "$V: $(tail -1 $O/${T}_pytest_$V.log)"; [ $rc -eq 0 ] || exit $rc
done
for V in libbshot_amd ab/libbshot_nw6w6 ab/libbshot_nw5w5 ab/libbshot_nw4w5 ab/libbshot_nw16 libbshot_amd ab/libbshot_nw6w6 ab/libbshot_nw5w5 ab/libbshot_nw4w5 ab/libbshot_nw16; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_nw6w6.so $L/ab/libbshot_nw5w5.so $L/ab/libbshot_nw4w5.so $L/ab/libbshot_nw16.so | tee $O/${T}_ab.txt || exit 1
