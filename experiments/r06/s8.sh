#!/bin/bash
# round 6 session 8: ICP release relayed in device memory (icp_relay 1) vs every workgroup polling host memory
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06h}
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "icp or odometry_hdl64_k2048 or lookahead" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
rm -f $O/abo_*
BENCH_INTERVALS=1 bash experiments/quick/ab_opts.sh 3 default icp_relay=0 | tee $O/${T}_ab.txt || exit 1
python experiments/r06/icp_tail.py $O/abo_default_*.err $O/abo_icp_relay_0_*.err > $O/${T}_icp_tail.txt
grep -h "grid searches per sweep\|\[0, 5\|\[60" $O/${T}_icp_tail.txt
python experiments/r05/icp_waits.py $O/abo_default_*.err $O/abo_icp_relay_0_*.err | grep -v "p75\|p99"
