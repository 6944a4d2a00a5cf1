# host timeline of the 7-simulated-peer exchange run (BSHOT_HOST_TRACE marks, no profiler)
mkdir -p gpurun_out
BSHOT_HOST_TRACE=gpurun_out/host_sim7.csv timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg --sim-peers 7 --steps 100 --warmup 10 > gpurun_out/sim7t.json 2> gpurun_out/sim7t.err || { tail -5 gpurun_out/sim7t.err; exit 1; }
python b-shot-slam_amd/tools/host_phases.py gpurun_out/host_sim7.csv
