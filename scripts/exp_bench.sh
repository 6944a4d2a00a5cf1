#!/bin/bash
# bench lines only (no tests): each argument is one set of extra bench.py flags (quoted)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
# an argument "@<lib> <flags>" runs that diagnostic build (make variant) through BSHOT_LIB
for args in "$@"; do
  lib=""
  if [ "${args:0:1}" = "@" ]; then lib=${args%% *}; lib=${lib:1}; args=${args#"@$lib"}; fi
  BSHOT_LIB=${lib:+$R/$lib} timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/eb.json 2> gpurun_out/eb.err || { tail -5 gpurun_out/eb.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/eb.json')); print(sys.argv[1] or '-', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_ms_per_sweep'], 'corr', d['config'].get('mutual_corr'))" "${lib}${args}"
done
