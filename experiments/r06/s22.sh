#!/bin/bash
# round 6 session 22: the s21 A/B in the reverse order (dp0 first), 4 rounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06w}
L=b-shot-slam_amd/lib
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 4 $L/ab/libbshot_dp0.so $L/libbshot_amd.so | tee $O/${T}_ab.txt || exit 1
