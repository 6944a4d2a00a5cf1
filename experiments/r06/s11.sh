#!/bin/bash
# round 6 session 11: SR run length vs the main stream's ICP iteration-0 wait (longer SR waves hold CUs
# the latency-critical ICP lists kernel waits for)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06k}
rm -f $O/abo_*
BENCH_INTERVALS=1 bash experiments/quick/ab_opts.sh 3 sr_run=1 sr_run=2 default iss_xcd_chunk=0 | tee $O/${T}_ab.txt || exit 1
python experiments/r05/icp_waits.py $O/abo_sr_run_1_*.err $O/abo_sr_run_2_*.err $O/abo_default_*.err $O/abo_iss_xcd_chunk_0_*.err | grep -v "p75\|p99\|corr" | tee $O/${T}_icp_waits.txt
