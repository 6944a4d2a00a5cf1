#!/bin/bash
# round 6 session 31: HEAD vs the r06p perf set's library (7dfb933) vs round 5's, same box, 200-sweep
# and driver-sized (20-sweep) lines
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zi}
L=b-shot-slam_amd/lib
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_r6p.so $L/ab/libbshot_r5.so | tee $O/${T}_ab.txt || exit 1
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/ab/libbshot_r5.so $L/ab/libbshot_r6p.so $L/libbshot_amd.so -- --steps 20 --warmup 5 | tee $O/${T}_ab_driver.txt || exit 1
