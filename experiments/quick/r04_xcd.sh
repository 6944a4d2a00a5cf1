#!/bin/bash
# SR XCD-local chunks: parity, standalone SR per chunk size (+ FETCH_SIZE), then a bench A/B of option sets
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "seg_ratio or golden or gmap or odometry or xchg or map" > $O/r04_xcd_pytest.log 2>&1
rc=$?; tail -3 $O/r04_xcd_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python b-shot-slam_amd/tools/sr_bench.py default sr_xcd_chunk=512 sr_xcd_chunk=1024 sr_xcd_chunk=2048 sr_xcd_chunk=4096 sr_xcd_chunk=0 || exit 1
cd /tmp && export TMPDIR=/tmp
for Z in 0 1024 4096; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/xcd_fetch_$Z -o f --output-format csv -- python3 $R/b-shot-slam_amd/tools/sr_bench.py sr_xcd_chunk=$Z > $O/xcd_fetch_$Z.log 2>&1 || exit 1
  python3 - $O/xcd_fetch_$Z <<'PY'
import csv, glob, sys, statistics
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_seg_ratio<false>" in r["Kernel_Name"]]
print(sys.argv[1].rsplit("_", 1)[1], "FETCH_SIZE KiB median", statistics.median(v), "n", len(v))
PY
done
cd $R
bash experiments/quick/ab_opts.sh ${1:-2} default sr_xcd_chunk=1024 sr_xcd_chunk=4096
