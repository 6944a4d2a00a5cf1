set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread -k "ransac" > $O/q1_pytest.log 2>&1; rc=$?; tail -3 $O/q1_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/q1_bench$i.json 2>$O/q1_bench$i.err || exit 1; cat $O/q1_bench$i.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_ms_per_sweep'])"
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q1_drv$i.json 2>$O/q1_drv$i.err || exit 1; cat $O/q1_drv$i.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_ms_per_sweep'])"; grep sweep_intervals $O/q1_drv$i.err
done
