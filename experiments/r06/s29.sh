#!/bin/bash
# round 6 session 29 (s28 with the target rows reserved in the pipeline path too): the GPU map and the matcher's target rows reserved up front (gmap_slots0 2^20,
# 2^18 target rows) vs the map doubling from 2 Ki slots (gmap_slots0=2048): map tests, the regrowth
# trace of a driver-sized bench, driver-sized (20 sweeps) and 200-sweep A/Bs
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zg}
timeout -k 10 500 python -u -m pytest tests/test_gmap_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
BSHOT_GROW_TRACE=1 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${T}_grow.json 2> $O/${T}_grow.err || exit 1
python3 - "$O/${T}_grow.err" <<'PY' | tee $O/${T}_grow.txt
import json, re, sys
err = open(sys.argv[1]).read().splitlines()
d = json.loads([x for x in err if x.startswith('{"sweep')][0])
t0, end = d['t0_ms'], d['marks_ms'][-1]
ev = [(float(m.group(1)), m.group(2)) for m in (re.match(r'\[bshot grow\] t=([\d.]+) ms (.*)', x) for x in err) if m]
inside = [(round(t - t0, 3), k) for t, k in ev if t0 <= t <= end]
print("regrowth events:", len(ev), "inside the timed region:", len(inside), inside)
PY
rm -f $O/abo_*
bash experiments/quick/ab_opts.sh 4 default gmap_slots0=2048 -- --steps 20 --warmup 5 | tee $O/${T}_ab_driver.txt || exit 1
