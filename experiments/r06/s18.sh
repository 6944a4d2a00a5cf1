#!/bin/bash
# round 6 session 18: config 3 and 5 lines with their own traces + PMC, the exchange with 7 simulated
# peers vs solo (as experiments/r05/round_final.sh without the perf part)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06s}
for P in 0 7; do
  if [ $P = 0 ]; then A="--no-map-bcast"; else A="--sim-peers $P"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A > $O/${T}_sim_$P.json 2> $O/${T}_sim_$P.err || { tail -5 $O/${T}_sim_$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${T}_sim_$P.json')); print('peers $P', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'], d['config']['parallelism'])" | tee -a $O/${T}_sim_peers.txt
done
bash scripts/gpu_config.sh ${T}_c3 --keypoints 600 --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash scripts/gpu_config.sh ${T}_c5 --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
