#!/bin/bash
# round 6 session 7: ICP iteration workgroups with helper waves for the grid searches (ICPH_WAVES 4
# product vs 1 / 2 / 8) -- ICP + odometry tests on the product and w8, alternating benches with
# per-sweep ICP tails
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06g}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or odometry or seg_ratio_point or sequence" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
BSHOT_LIB=$R/$L/ab/libbshot_w8.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "icp" > $O/${T}_pytest_w8.log 2>&1
rc=$?; echo "w8: $(tail -1 $O/${T}_pytest_w8.log)"; [ $rc -eq 0 ] || exit $rc
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_w1.so $L/ab/libbshot_w2.so $L/ab/libbshot_w8.so | tee $O/${T}_ab.txt || exit 1
for V in amd w1 w2 w8; do python experiments/r06/icp_tail.py $O/abm_libbshot_${V}_*.err; done > $O/${T}_icp_tail.txt
grep -h "grid searches per sweep\|\[60" $O/${T}_icp_tail.txt
