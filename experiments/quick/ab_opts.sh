#!/bin/bash
# A/B/C... of option sets on one library, alternating: usage ab_opts.sh <rounds> <set>... [-- bench args]
# a set is "name=value,name=value" or "default"; prints per run: set, round, sweeps/s, median ms,
# main-thread host phases, SR stage ms
N=$1; shift
SETS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done; [ "${1:-}" = "--" ] && shift
O=gpurun_out; mkdir -p $O
for i in $(seq 1 $N); do for S in "${SETS[@]}"; do
  T=$(echo "$S" | tr ',=' '__')
  A=(); if [ "$S" != default ]; then IFS=',' read -ra KV <<< "$S"; for kv in "${KV[@]}"; do A+=(--opt "$kv"); done; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg "${A[@]}" "$@" > $O/abo_${T}_$i.json 2> $O/abo_${T}_$i.err || { tail -5 $O/abo_${T}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/abo_${T}_$i.json'))
print('$S', $i, d['value'], d['ms_per_step_median'], {k: round(v, 3) for k, v in d.get('host_ms_per_sweep', {}).items()}, d.get('stage_ms_per_sweep', {}).get('seg_ratio'))"
done; done
