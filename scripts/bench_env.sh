#!/bin/bash
# bench lines under different environment settings: bash scripts/bench_env.sh "" "GPU_MAX_HW_QUEUES=8" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
i=0
for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --steps ${STEPS:-40} ${BENCH_ARGS:-} > gpurun_out/be_$i.json 2> gpurun_out/be_$i.err || { tail -5 gpurun_out/be_$i.err; exit 1; }
    python3 - "$e" gpurun_out/be_$i.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().splitlines()[0])
E = [l for l in open(sys.argv[2][:-5] + ".err").read().splitlines() if l.startswith('{"host_ms')]
h = json.loads(E[-1])["host_ms_per_sweep"] if E else {}
print(f"{sys.argv[1]:40s} {b['value']:8.1f} sweeps/s  host {h}")
PY
done
