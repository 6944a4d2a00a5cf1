#!/bin/bash
# round 6 session 4: ISS PMC by XCD chunking (separate counter passes), pipeline A/B of the SR runs / ISS chunks
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06d}
cd /tmp && export TMPDIR=/tmp
for X in 0 1024; do
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/${T}_pmcf_iss$X -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/iss_bench.py iss_xcd_chunk=$X > $O/${T}_pmcf_iss$X.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/${T}_pmch_iss$X -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/iss_bench.py iss_xcd_chunk=$X > $O/${T}_pmch_iss$X.log 2>&1 || exit 1
done
cd $R && python3 - <<PY
import csv, glob, collections
for X in (0, 1024):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for d in ("pmcf", "pmch"):
        f = glob.glob("$O/${T}_%s_iss%d/**/*counter_collection.csv" % (d, X), recursive=True)
        for r in csv.DictReader(open(f[0])):
            k = r["Kernel_Name"]
            if "iss" not in k: continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
    for k, dd in agg.items():
        m = {c: v / n[(k, c)] for c, v in dd.items()}
        hit = m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0))
        print(X, k[:40], "fetch MB/launch %.1f" % (m.get("FETCH_SIZE", 0) * 2 / 1024), "L2 hit %.3f" % hit)
PY
rm -rf $O/${T}_pmc?_iss*
bash experiments/quick/ab_opts.sh 2 sr_run=1,iss_xcd_chunk=0 default sr_run=4,iss_xcd_chunk=0 | tee $O/${T}_ab.txt
