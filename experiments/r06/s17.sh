#!/bin/bash
# round 6 session 17: ISS lane kernel with 16 keys in registers (8 KB LDS, 122 VGPRs, 4 waves/SIMD;
# product) vs all keys in LDS (rk0 = HEAD) vs register keys with the wide batches (rkc8, 154 VGPRs):
# ISS parity, standalone ISS, alternating benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06r}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "iss or golden or keypoint" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
BSHOT_LIB=$R/$L/ab/libbshot_rkc8.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "iss" > $O/${T}_pytest_rkc8.log 2>&1
rc=$?; echo "rkc8: $(tail -1 $O/${T}_pytest_rkc8.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_rk0 ab/libbshot_rkc8 libbshot_amd ab/libbshot_rk0 ab/libbshot_rkc8; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/iss_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_iss_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_rk0.so $L/ab/libbshot_rkc8.so | tee $O/${T}_ab.txt || exit 1
