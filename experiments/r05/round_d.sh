#!/bin/bash
# round 5 session d: full GPU suite (fused ladder build, counted ICP grids, ICP loop staging), then the ICP A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r05d}
bash scripts/gpu_round.sh $T tests || exit 1
bash experiments/r05/icp_ab.sh $T 2
