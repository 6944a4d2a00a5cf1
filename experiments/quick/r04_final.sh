#!/bin/bash
# Round-4 final set on HEAD: GPU suite + smoke + perf (gpu_round), exchange with 7 simulated peers,
# config-3 and config-5 lines with their own profiles
set -u
TAG=${1:-r04d}
O=gpurun_out; mkdir -p $O
bash scripts/gpu_round.sh $TAG all || exit 1
for P in 0 7; do
  if [ $P = 0 ]; then A="--no-map-bcast"; else A="--sim-peers $P"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A > $O/${TAG}_sim_$P.json 2> $O/${TAG}_sim_$P.err || { tail -5 $O/${TAG}_sim_$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_sim_$P.json')); print('peers $P', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'], d['config']['parallelism'])" | tee -a $O/${TAG}_sim_peers.txt
done
bash scripts/gpu_config.sh ${TAG}_c3 --keypoints 600 --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash scripts/gpu_config.sh ${TAG}_c5 --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
