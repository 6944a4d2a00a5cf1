#!/bin/bash
# round 6 session 30: final perf set on HEAD (bench, driver-sized, host timeline, kernel trace, PMC),
# the regrowth trace of the default 200-sweep bench, config 3 and 5 lines with their own traces + PMC
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zh}
bash scripts/gpu_round.sh $T perf || exit 1
cd $R
BSHOT_GROW_TRACE=1 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-upload-leg > $O/${T}_grow200.json 2> $O/${T}_grow200.err || exit 1
python3 - "$O/${T}_grow200.err" <<'PY' | tee $O/${T}_grow200.txt
import json, re, sys
err = open(sys.argv[1]).read().splitlines()
d = json.loads([x for x in err if x.startswith('{"sweep')][0])
t0, end = d['t0_ms'], d['marks_ms'][-1]
ev = [(float(m.group(1)), m.group(2)) for m in (re.match(r'\[bshot grow\] t=([\d.]+) ms (.*)', x) for x in err) if m]
inside = [(round(t - t0, 3), k) for t, k in ev if t0 <= t <= end]
print("200-sweep region: regrowth events", len(ev), "inside:", len(inside), inside)
PY
bash scripts/gpu_config.sh ${T}_c3 --keypoints 600 --steps 1000 --warmup 20 --no-cpu-baseline || exit 1
bash scripts/gpu_config.sh ${T}_c5 --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 --no-cpu-baseline
