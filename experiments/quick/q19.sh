set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3 4 5 6; do for v in def blit; do
E="BSHOT_X=0"; [ $v = blit ] && E="GPU_FORCE_BLIT_COPY_SIZE=256"
env $E BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q19_$v$i.json 2>$O/q19_$v$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q19_$v$i.json')); e=[json.loads(l) for l in open('$O/q19_$v$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print('$v', d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)))"
done; done
env GPU_FORCE_BLIT_COPY_SIZE=256 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/q19_long_blit.json 2>/dev/null && python3 -c "import json; d=json.load(open('$O/q19_long_blit.json')); print('long blit', d['value'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/q19_long_def.json 2>/dev/null && python3 -c "import json; d=json.load(open('$O/q19_long_def.json')); print('long def', d['value'])"
