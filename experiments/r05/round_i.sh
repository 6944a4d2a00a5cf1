#!/bin/bash
# round 5 session i: GPU suite + smoke on HEAD, then config 3 and config 5 lines with their own traces + PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r05i}
bash scripts/gpu_round.sh $T tests || exit 1
bash scripts/gpu_config.sh ${T}_c3 --keypoints 600 --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash scripts/gpu_config.sh ${T}_c5 --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
