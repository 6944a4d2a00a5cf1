#!/bin/bash
# SR parity tests, standalone SR (base vs tree), then an A/B of bench lines
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
N=${1:-2}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "seg_ratio or golden or parity or iss or describe or normals" > $O/r04_sr2_pytest.log 2>&1
rc=$?; tail -3 $O/r04_sr2_pytest.log; [ $rc -eq 0 ] || exit $rc
for L in experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so ${EXTRA_LIBS:-}; do
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py || exit 1
done
bash experiments/quick/ab_multi.sh $N experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so ${EXTRA_LIBS:-}
