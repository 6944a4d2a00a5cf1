#!/bin/bash
# round 6 session 15: pipelined centroid sums (product) vs the previous seq_sum (ss0): SR/normals parity,
# standalone SR, alternating benches
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06o}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -k "seg_ratio or normals or describe or golden" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_ss0 libbshot_amd ab/libbshot_ss0; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py | sed "s|^|$V |"; done | tee $O/${T}_sr_bench.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_ss0.so | tee $O/${T}_ab.txt || exit 1
