#!/bin/bash
# round 5 session i: GPU suite + smoke on HEAD, then config 3 and config 5 lines with their own traces + PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
T=${1:-r05i}
bash scripts/gpu_round.sh $T tests || exit 1
# (config 3 measured in the final set)
bash scripts/gpu_config.sh ${T}_c5 --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
# config 5: the histogram / rank_wg kernels in LPT slices (option desc_slices) vs one launch each
O=$R/gpurun_out
for i in 1 2; do for S in 1 4; do
  timeout -k 10 300 python bench.py --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline --no-upload-leg --opt desc_slices=$S > $O/${T}_c5s$S.json 2> $O/${T}_c5s$S.err || exit 1
  python3 -c "import json; d=json.load(open('$O/${T}_c5s$S.json')); print('desc_slices $S', $i, d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'])" | tee -a $O/${T}_c5_slices.txt
done; done
# ISS: a lane's cell scan 8 points per round trip (product) vs 4 (libbshot_scan4)
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 2 b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_scan4.so | tee $O/${T}_ab_iss_scan.txt
