# experiment: the map insert's LDS image cut to 1024 members (GM_LDS_N): does the 7-peer period move?
mkdir -p gpurun_out
for P in 0 7 0 7; do
  if [ $P = 0 ]; then A="--no-map-bcast"; else A="--sim-peers $P"; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A > gpurun_out/siml_$P.json 2> gpurun_out/siml_$P.err || { tail -5 gpurun_out/siml_$P.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/siml_$P.json')); print('peers $P', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'])"
done
