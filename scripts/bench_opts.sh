#!/bin/bash
# bench lines for several option sets: bash scripts/bench_opts.sh "--opt a=1" "--opt a=2 --depth 1" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
i=0
for o in "$@"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages --steps ${STEPS:-40} $o > gpurun_out/bo_$i.json 2> gpurun_out/bo_$i.err || { tail -5 gpurun_out/bo_$i.err; exit 1; }
    python3 - "$o" gpurun_out/bo_$i.json <<'PY'
import json, sys
b = json.loads(open(sys.argv[2]).read().splitlines()[0])
E = [l for l in open(sys.argv[2][:-5] + ".err").read().splitlines() if l.startswith('{"host_ms')]
h = json.loads(E[-1])["host_ms_per_sweep"] if E else {}
print(f"{sys.argv[1]:40s} {b['value']:8.1f} sweeps/s  host {h}")
PY
done
