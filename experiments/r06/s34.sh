#!/bin/bash
# round 6 session 34: the describe (side) stream's priority re-measured on HEAD (round 4: higher was slower)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zn}
rm -f $O/abo_*
bash experiments/quick/ab_opts.sh 3 default side_prio=1 side_prio=2 | tee $O/${T}_ab_side_prio.txt || exit 1
