set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4 5 6; do
s=$(date +%s.%N)
HIP_ENABLE_DEFERRED_LOADING=0 BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q11_$i.json 2>$O/q11_$i.err || exit 1
python3 -c "
import json,time; d=json.load(open('$O/q11_$i.json')); e=[json.loads(l) for l in open('$O/q11_$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print(d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)), 'wall %.1f s' % (time.time()-$s))"
done
