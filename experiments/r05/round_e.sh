#!/bin/bash
# round 5 session e: full GPU suite (launch diet: fused ladder tables, counted ICP grids, paired copies),
# counted vs sorted ICP grids bench A/B, kernel trace of the product build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05e}
bash scripts/gpu_round.sh $T tests || exit 1
MODES="host hostsg" bash experiments/r05/icp_ab.sh $T 2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T} -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}.json 2> $O/prof_${T}.err
