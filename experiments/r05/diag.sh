#!/bin/bash
# marginal cost of stages: bench lines of diagnostic builds (results not valid) against the tree
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
E=b-shot-slam_amd/lib/exp
for i in 1 2; do
for L in $E/libbshot_topk.so $E/libbshot_nofin.so $E/libbshot_hfnoap.so $E/libbshot_hfnorec.so; do
  BSHOT_LIB=$R/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg > $O/diag.json 2> $O/diag.err || { tail -3 $O/diag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/diag.json')); print('$(basename $L .so)', d['value'], d['ms_per_step_median'], d['stage_ms_per_sweep'])"
done
BSHOT_LIB=$R/$E/libbshot_topk.so timeout -k 10 200 python experiments/quick/diag_param.py run_iss=0 --no-cpu-baseline --no-upload-leg > $O/diag.json 2> $O/diag.err || { tail -3 $O/diag.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/diag.json')); print('noiss', d['value'], d['ms_per_step_median'], d['stage_ms_per_sweep'])"
done
