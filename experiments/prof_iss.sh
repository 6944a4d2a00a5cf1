R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pi -o t --output-format csv -- python3 $R/experiments/iss_variants.py > $R/gpurun_out/pi.log 2>&1 || exit $?
python3 - "$R/gpurun_out/pi/t_kernel_stats.csv" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
