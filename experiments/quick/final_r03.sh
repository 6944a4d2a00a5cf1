set -u
# Round-3 final validation on HEAD: the GPU suite + smoke, a 1-rank RCCL exchange run with simulated
# peers (map_sync 0, the bench default), and the config-3 / config-5 lines with their profiles.
O=gpurun_out; mkdir -p $O
bash scripts/gpu_round.sh r03h tests || exit 1
echo "[final] $(date +%T) sim-peers exchange" &&
timeout -k 10 300 python bench.py --sim-peers 3 --steps 100 --warmup 10 --no-cpu-baseline --no-upload-leg > $O/r03h_sim_peers3.json 2> $O/r03h_sim_peers3.err &&
cat $O/r03h_sim_peers3.json &&
bash scripts/gpu_config.sh r03c3h --keypoints 600 --steps 1000 --warmup 20 --no-cpu-baseline &&
bash scripts/gpu_config.sh r03c5h --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
