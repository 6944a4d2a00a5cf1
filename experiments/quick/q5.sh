set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3; do for v in a b; do
X=""; [ $v = b ] && X="--no-stage-timing"
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 $X > $O/q5_$v$i.json 2>$O/q5_$v$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q5_$v$i.json')); e=[json.loads(l) for l in open('$O/q5_$v$i.err') if l.startswith('{\"sweep')][0]
print('$v', d['value'], d['ms_per_step'], e['sweep_intervals_ms'][:3])"
done; done
