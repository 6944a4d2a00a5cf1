set -u
# Standalone (uncontended) SR work counters + SR / describe kernel times on one HDL-64 sweep.
# usage: bash experiments/quick/r03_diag.sh [tag]   (BSHOT_LIB selects the library)
T=${1:-x}
O=gpurun_out; mkdir -p $O
R=$(pwd)
timeout -k 10 120 python b-shot-slam_amd/tools/knn_stats.py > $O/diag_knn_stats_$T.json 2>&1 && cat $O/diag_knn_stats_$T.json &&
timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py > $O/diag_describe_$T.json 2>&1 && cat $O/diag_describe_$T.json &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/$O/diag_prof_$T -o t --output-format csv -- \
    python3 $R/b-shot-slam_amd/tools/describe_bench.py > $R/$O/diag_prof_$T.log 2>&1 &&
cd $R && python3 - $T <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/diag_prof_{sys.argv[1]}/**/t_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if float(r['AverageNs']) > 15000: print(sys.argv[1], r['Name'][:40], r['Calls'], round(float(r['AverageNs']) / 1000, 1))
PY
