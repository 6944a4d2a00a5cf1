set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4; do
BSHOT_GROW_TRACE=1 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q6_$i.json 2>$O/q6_$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q6_$i.json')); e=[json.loads(l) for l in open('$O/q6_$i.err') if l.startswith('{\"sweep')][0]
print(d['value'], d['ms_per_step'], e['sweep_intervals_ms'][:3], e['work'])"
grep -c "grow\] .*device" $O/q6_$i.err
done
