#!/bin/bash
# round 6 session 26: SHOT records' divisions by the constants R/2, 90 and 45 degrees as reciprocal +
# two FMAs (product) vs IEEE division (dv0): describe / odometry parity, standalone describe,
# alternating benches (both orders) and config 5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06za}
L=b-shot-slam_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or shot or golden or config5 or lookahead or replay or sequence" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_dv0 libbshot_amd ab/libbshot_dv0; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_dv0.so | tee $O/${T}_ab.txt || exit 1
bash experiments/quick/ab_multi.sh 3 $L/ab/libbshot_dv0.so $L/libbshot_amd.so | tee $O/${T}_ab_rev.txt || exit 1
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_dv0.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_c5.txt || exit 1
