#!/bin/bash
# describe A/B: parity subset for each lib, standalone describe stages, then alternating bench lines
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
N=$1; K=$2; shift 2
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
for L in "${LIBS[@]}"; do
  if [ "$K" != "-" ]; then
    BSHOT_LIB=$R/$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/ab_pytest_$(basename $L .so).log 2>&1
    rc=$?; echo "$(basename $L) tests: $(tail -1 $O/ab_pytest_$(basename $L .so).log)"; [ $rc -eq 0 ] || exit $rc
  fi
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | tail -3 | sed "s|^|$(basename $L .so) |" || exit 1
done
[ $N -gt 0 ] && bash experiments/quick/ab_multi.sh $N "${LIBS[@]}" -- "$@"
