#!/bin/bash
# round 6 session 20: standalone per-kernel split of ISS, SR and describe (kernel trace of the
# stage benches, no pipeline beside them)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
T=${1:-r06u}
for B in iss_bench sr_bench describe_bench; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_${T}_$B -o t --output-format csv -- python3 $R/b-shot-slam_amd/tools/$B.py > $O/${T}_$B.log 2>&1 || { echo "$B failed"; tail -5 $O/${T}_$B.log; exit 1; }
  f=$(find $O/p_${T}_$B -name "t_kernel_stats.csv" | head -1); cp $f $O/${T}_${B}_kernel_stats.csv; rm -rf $O/p_${T}_$B
  echo "== $B"; python3 -c "
import csv
for r in list(csv.DictReader(open('$O/${T}_${B}_kernel_stats.csv')))[:12]:
    print('  %-60s %6s %9.1f us %s' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, r['Percentage']))"
done
