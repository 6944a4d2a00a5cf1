#!/bin/bash
# round 6 session 9: ladder sort with 4096 / 2048 keys per rocprim block (fewer merge passes) vs the
# default 1024; then a kernel trace of the product bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06i}
L=b-shot-slam_amd/lib
BSHOT_LIB=$R/$L/ab/libbshot_b4k.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "seg_ratio or iss or icp_exact" > $O/${T}_pytest_b4k.log 2>&1
rc=$?; echo "b4k: $(tail -1 $O/${T}_pytest_b4k.log)"; [ $rc -eq 0 ] || exit $rc
for V in amd ab/libbshot_hd1 ab/libbshot_hd2; do
  F=$L/$V.so; [ "$V" = amd ] && F=$L/libbshot_amd.so
  BSHOT_LIB=$R/$F timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1
done | tee $O/${T}_describe_diag.txt
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_b4k.so $L/ab/libbshot_b2k.so | tee $O/${T}_ab_sort.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/${T}_prof -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg > $O/${T}_prof_bench.json 2> $O/${T}_prof_bench.err || exit 1
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/${T}_kernel_stats.csv; head -32 "$f" | cut -d, -f1-4 | cut -c1-150; rm -rf $O/${T}_prof
