set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4 5; do
BSHOT_HOST_TRACE=$O/q7_host$i.csv BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q7_$i.json 2>$O/q7_$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q7_$i.json')); e=[json.loads(l) for l in open('$O/q7_$i.err') if l.startswith('{\"sweep')][0]
print(d['value'], d['ms_per_step'], e['sweep_intervals_ms'][:3])"
done
