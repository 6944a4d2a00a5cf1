O=gpurun_out
for i in 1 2; do
for v in skip run; do
  E=""; [ $v = skip ] && E="--opt diag_skip_icp=1"
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg $E > $O/noicp_$v$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/noicp_$v$i.json')); print('$v', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'])"
done; done
