# the map exchange's per-sweep insert cost on the period, on one GPU:
# a 1-rank RCCL exchange plus P simulated peers' replica inserts (bench.py --sim-peers), P = 0..7
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_xchg_gpu.py tests/test_gmap_gpu.py tests/test_multiseq_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_sim.log 2>&1 || { tail -30 gpurun_out/pt_sim.log; exit 1; }
tail -1 gpurun_out/pt_sim.log
for P in 0 7 0 7 3; do
  if [ $P = 0 ]; then A="--no-map-bcast"; else A="--sim-peers $P"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A > gpurun_out/sim_$P.json 2> gpurun_out/sim_$P.err || { tail -5 gpurun_out/sim_$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/sim_$P.json')); print('peers $P', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'], d['config']['parallelism'])"
done
BSHOT_HOST_TRACE=gpurun_out/host_sim7.csv timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg --sim-peers 7 --steps 100 --warmup 10 > gpurun_out/sim7t.json 2> gpurun_out/sim7t.err || { tail -5 gpurun_out/sim7t.err; exit 1; }
python b-shot-slam_amd/tools/host_phases.py gpurun_out/host_sim7.csv
