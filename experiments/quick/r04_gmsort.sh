#!/bin/bash
# map-insert sort kernel: GPU map / odometry / exchange tests, then the hist_fused diagnostics
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gmap or odometry or xchg or sequence or map" > $O/r04_gmsort_pytest.log 2>&1
rc=$?; tail -3 $O/r04_gmsort_pytest.log; [ $rc -eq 0 ] || exit $rc
bash experiments/quick/r04_hfdiag.sh
