cd $GRAFT_REPO_ROOT
for args in "" "--no-stage-timing" "--opt queue_thread=1" "--no-stage-timing --opt queue_thread=1" "" "--no-stage-timing"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 20 $args | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$args', d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'])" || exit 1
done
