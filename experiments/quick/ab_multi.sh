#!/bin/bash
# A/B/C... of library builds on one box, alternating: usage ab_multi.sh <rounds> <lib>... [-- bench args]
# prints per run: lib, round, sweeps/s, median ms/step, main-thread host phases, SR stage ms
N=$1; shift
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
O=gpurun_out; mkdir -p $O
for i in $(seq 1 $N); do for L in "${LIBS[@]}"; do
  T=$(basename $L .so)
  BSHOT_LIB=$(pwd)/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg "$@" > $O/abm_${T}_$i.json 2> $O/abm_${T}_$i.err || { tail -5 $O/abm_${T}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/abm_${T}_$i.json'))
print('$T', $i, d['value'], d['ms_per_step_median'], {k: round(v, 3) for k, v in d.get('host_ms_per_sweep', {}).items()}, d.get('stage_ms_per_sweep', {}).get('seg_ratio'))"
done; done
