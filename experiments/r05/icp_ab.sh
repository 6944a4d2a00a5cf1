#!/bin/bash
# round 5: ICP loop A/B -- ICP parity tests on the product build, then alternating bench lines:
# host loop (default) vs the device loop (icp_device 1) in the product build and two variants
# usage: icp_ab.sh <tag> [rounds] [extra bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=$1; N=${2:-2}; shift 2 || true
L=b-shot-slam_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "icp" > $O/${T}_icp_pytest.log 2>&1
rc=$?; tail -2 $O/${T}_icp_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq $N); do
  for M in ${MODES:-host dev devold hostsg}; do
    case $M in
      host) LIB=$L/libbshot_amd.so; A="";;
      dev) LIB=$L/libbshot_amd.so; A="--opt icp_device=1";;
      devold) LIB=$L/exp/libbshot_icpold.so; A="--opt icp_device=1";;
      hostsg) LIB=$L/exp/libbshot_sgrid.so; A="";;
    esac
    BSHOT_LIB=$R/$LIB timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A "$@" > $O/${T}_$M.json 2> $O/${T}_$M.err || { tail -5 $O/${T}_$M.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${T}_$M.json')); print('$M', $i, d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'])" | tee -a $O/${T}_icp_ab.txt
  done
done
