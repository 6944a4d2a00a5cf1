#!/bin/bash
# round 6 session 27: ISS lane kernel skipping the cube cells whose box lies beyond the radius
# (product) vs every cube cell (pr0): ISS parity, standalone ISS kernels, benches (both orders)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06zc}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "iss or golden or keypoint" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for V in libbshot_amd ab/libbshot_pr0 libbshot_amd ab/libbshot_pr0; do
  N=$(basename $V)
  BSHOT_LIB=$R/$L/$V.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_${T}_$N -o t --output-format csv -- python3 $R/b-shot-slam_amd/tools/iss_bench.py > $O/${T}_iss_$N.log 2>&1 || { echo "$V failed"; exit 1; }
  f=$(find $O/p_${T}_$N -name "t_kernel_stats.csv" | head -1)
  echo "$V $(grep '^{' $O/${T}_iss_$N.log | cut -c1-200)"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'k_iss' in r['Name']: print('   %-28s %9.1f us' % (r['Name'][:28], float(r['AverageNs'])/1e3))"
  rm -rf $O/p_${T}_$N
done | tee $O/${T}_iss_bench.txt
cd $R
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_pr0.so | tee $O/${T}_ab.txt || exit 1
bash experiments/quick/ab_multi.sh 3 $L/ab/libbshot_pr0.so $L/libbshot_amd.so | tee $O/${T}_ab_rev.txt || exit 1
