#!/bin/bash
# round 6 session 5: per-sweep ICP tail vs grid searches; hash-table size sensitivity (diagnostic builds)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06e}
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-upload-leg > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cat $O/${T}_bench.json | head -c 600; echo
python experiments/r06/icp_tail.py $O/${T}_bench.err | tee $O/${T}_icp_tail.txt
L=b-shot-slam_amd/lib
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_h17.so $L/ab/libbshot_h16.so | tee $O/${T}_ab_tables.txt
