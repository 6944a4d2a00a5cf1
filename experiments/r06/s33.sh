#!/bin/bash
# round 6 session 33: describe-chain workgroups sized to fit beside SR's (k_shot_rank in 1-wave
# workgroups, 2 KB of LDS: product) vs 4-wave ones (srk4, 8 KB) vs product + 2-wave k_lrf_eig
# workgroups (le2, 6 KB instead of 12): describe parity, standalone describe, benches both orders
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zl}
L=b-shot-slam_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or shot or golden or config5" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
BSHOT_LIB=$R/$L/ab/libbshot_le2.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe_parity or describe_device_plan" > $O/${T}_pytest_le2.log 2>&1
rc=$?; echo "le2: $(tail -1 $O/${T}_pytest_le2.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_srk4 ab/libbshot_le2 libbshot_amd ab/libbshot_srk4 ab/libbshot_le2; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_srk4.so $L/ab/libbshot_le2.so | tee $O/${T}_ab.txt || exit 1
bash experiments/quick/ab_multi.sh 3 $L/ab/libbshot_le2.so $L/ab/libbshot_srk4.so $L/libbshot_amd.so | tee $O/${T}_ab_rev.txt || exit 1
