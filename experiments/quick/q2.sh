set -u
O=gpurun_out; mkdir -p $O
for i in 1 2; do
BSHOT_GROW_TRACE=1 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q2_drv$i.json 2>$O/q2_drv$i.err || exit 1; cat $O/q2_drv$i.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_ms_per_sweep'])"; grep -c "bshot grow" $O/q2_drv$i.err
done
