set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4 5 6; do for v in sdma0 def; do
E=""; [ $v = sdma0 ] && E="HSA_ENABLE_SDMA=0"
env $E BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q17_$v$i.json 2>$O/q17_$v$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q17_$v$i.json')); e=[json.loads(l) for l in open('$O/q17_$v$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print('$v', d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)))"
done; done
