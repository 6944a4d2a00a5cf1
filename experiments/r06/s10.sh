#!/bin/bash
# round 6 session 10: ISS overflow list as (point, position) pairs + non-max counts by position (tests,
# standalone); round 5's library vs HEAD on one box (alternating benches, kernel traces of both)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06j}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "iss or edge or odometry_hdl64_k600 or kp_test" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python b-shot-slam_amd/tools/iss_bench.py iss_xcd_chunk=0 iss_xcd_chunk=1024 iss_xcd_chunk=0 iss_xcd_chunk=1024 | tee $O/${T}_iss_bench.txt || exit 1
BSHOT_LIB=$R/$L/ab/libbshot_r5.so timeout -k 10 200 python b-shot-slam_amd/tools/iss_bench.py | sed 's/^/r5 /' | tee -a $O/${T}_iss_bench.txt || exit 1
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_r5.so | tee $O/${T}_ab_r5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for V in amd r5; do
  F=$R/$L/libbshot_amd.so; [ $V = r5 ] && F=$R/$L/ab/libbshot_r5.so
  BSHOT_LIB=$F timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/${T}_prof_$V -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg > $O/${T}_prof_bench_$V.json 2> $O/${T}_prof_bench_$V.err || exit 1
  f=$(find $O/${T}_prof_$V -name "*kernel_stats.csv" | head -1); cp "$f" $O/${T}_kernel_stats_$V.csv; rm -rf $O/${T}_prof_$V
done
