#!/bin/bash
# round 6 session 32: SR run length and bounded-pass grid ratio re-tuned on HEAD (options)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zk}
rm -f $O/abo_*
bash experiments/quick/ab_opts.sh 3 default sr_run=3 sr_run=6 sr_run=8 sr_bratio=150 sr_bratio=283 | tee $O/${T}_ab_sr.txt || exit 1
