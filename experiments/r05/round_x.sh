#!/bin/bash
# round 5 closing set on HEAD: GPU suite + smoke, then the final perf set (round_final.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r05x}
bash scripts/gpu_round.sh $T tests || exit 1
bash experiments/r05/round_final.sh $T
