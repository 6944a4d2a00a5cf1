#!/bin/bash
# round 5: exchange tests, then solo vs --sim-peers 7 (eager replicas, default) vs 7 lazy, alternating
# usage: xchg.sh <tag> [rounds]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=$1; N=${2:-2}
timeout -k 10 600 python -u -m pytest tests/test_xchg_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/${T}_xchg_pytest.log 2>&1
rc=$?; tail -3 $O/${T}_xchg_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq $N); do
  for M in solo eager7 lazy7; do
    case $M in
      solo) A="--no-map-bcast";;
      eager7) A="--sim-peers 7";;
      lazy7) A="--sim-peers 7 --xchg-lazy";;
    esac
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $A > $O/${T}_$M.json 2> $O/${T}_$M.err || { tail -5 $O/${T}_$M.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${T}_$M.json')); print('$M', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'], d['config']['parallelism'])" | tee -a $O/${T}_sim_peers.txt
  done
done
