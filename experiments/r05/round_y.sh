#!/bin/bash
# round 5 session y: option iss_defer (the queued sweep's ISS launched after the current sweep's ICP)
# vs default: lookahead parity tests, alternating bench A/B with per-sweep ICP waits
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05y}
timeout -k 10 300 python -u -m pytest tests/test_odometry_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lookahead" > $O/${T}_pytest.log 2>&1
rc=$?; tail -1 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/abo_*
BENCH_INTERVALS=1 bash experiments/quick/ab_opts.sh 3 default iss_defer=1 | tee $O/${T}_ab_iss_defer.txt || exit 1
python experiments/r05/icp_waits.py $O/abo_default_*.err $O/abo_iss_defer_1_*.err > $O/${T}_icp_waits.txt
