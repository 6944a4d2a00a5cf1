#!/bin/bash
# round 6 session 3: ISS XCD-local chunks + position-indexed lists (tests, standalone, PMC), SR run/bratio grid
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06c}
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py tests/test_edge_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "iss or odometry_hdl64_k600 or edge" > $O/${T}_pytest.log 2>&1
rc=$?; tail -3 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python b-shot-slam_amd/tools/iss_bench.py iss_xcd_chunk=0 iss_xcd_chunk=1024 iss_xcd_chunk=256 iss_xcd_chunk=4096 iss_xcd_chunk=0 iss_xcd_chunk=1024 > $O/${T}_iss_bench.txt 2>&1 || { cat $O/${T}_iss_bench.txt; exit 1; }
cat $O/${T}_iss_bench.txt
timeout -k 10 200 python b-shot-slam_amd/tools/sr_bench.py sr_run=1 sr_run=2 sr_run=3 sr_run=4 sr_run=2,sr_bratio=200 sr_run=3,sr_bratio=200 sr_run=4,sr_bratio=200 sr_run=6,sr_bratio=200 sr_run=1 > $O/${T}_sr_bench.txt 2>&1 || { cat $O/${T}_sr_bench.txt; exit 1; }
cat $O/${T}_sr_bench.txt
cd /tmp && export TMPDIR=/tmp
for X in 0 1024; do
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/${T}_pmc_iss$X -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/iss_bench.py iss_xcd_chunk=$X > $O/${T}_pmc_iss$X.log 2>&1 || exit 1
done
cd $R && python3 - <<PY
import csv, glob, collections
for X in (0, 1024):
    f = glob.glob("$O/${T}_pmc_iss%d/**/*counter_collection.csv" % X, recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "iss" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, d in agg.items():
        m = {c: v / n[(k, c)] for c, v in d.items()}
        hit = m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0))
        print(X, k[:40], "fetch MB/launch %.1f" % (m.get("FETCH_SIZE", 0) * 2 / 1024), "L2 hit %.3f" % hit)
PY
