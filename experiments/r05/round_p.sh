#!/bin/bash
# round 5 session p: k_shot_rank with the prefetched key window (product = libbshot_win) vs the 8-byte
# keys (libbshot_base = HEAD 0e1aa6c): describe parity tests, alternating bench A/B, kernel trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05p}
A=b-shot-slam_amd/lib/libbshot_amd.so; B=b-shot-slam_amd/lib/exp/libbshot_base.so
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "describe or rank or hist or sequence or chain" > $O/${T}_pytest.log 2>&1
rc=$?; tail -2 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $A $B | tee $O/${T}_ab_win.txt || exit 1
cd /tmp && export TMPDIR=/tmp
BSHOT_LIB=$R/$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T} -o trace --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}.json 2> $O/prof_${T}.err
