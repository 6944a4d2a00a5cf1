#!/bin/bash
# marginal cost of each big kernel: the tree against builds that run that kernel twice
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
E=b-shot-slam_amd/lib/exp
for i in 1 2; do
for L in $E/libbshot_tree.so $E/libbshot_sr2.so $E/libbshot_hf2.so $E/libbshot_iss2.so $E/libbshot_cnt2.so; do
  BSHOT_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg > $O/diag.json 2> $O/diag.err || { tail -3 $O/diag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/diag.json')); print('$(basename $L .so)', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['stage_ms_per_sweep'])"
done
done
