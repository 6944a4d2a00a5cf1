#!/bin/bash
# round 6 session 16: segment_normal sums pipelined in groups of 8 (product) vs the previous
# sequential loop (ln0): describe/normals parity, standalone describe, alternating benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06q}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or normal or golden or lrf" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_ln0 libbshot_amd ab/libbshot_ln0; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_ln0.so | tee $O/${T}_ab.txt || exit 1
