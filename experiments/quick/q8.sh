set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4 5 6; do
ROC_ACTIVE_WAIT_TIMEOUT=100000 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q8_$i.json 2>$O/q8_$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q8_$i.json')); e=[json.loads(l) for l in open('$O/q8_$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print(d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)))"
done
ROC_ACTIVE_WAIT_TIMEOUT=100000 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/q8_long.json 2>$O/q8_long.err || exit 1
python3 -c "import json; d=json.load(open('$O/q8_long.json')); print('long', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['host_ms_per_sweep'])"
