set -u
O=gpurun_out; mkdir -p $O
for i in 1 2 3; do for v in def blit cpdma; do
E="BSHOT_X=0"; [ $v = blit ] && E="GPU_FORCE_BLIT_COPY_SIZE=256"; [ $v = cpdma ] && E="GPU_CP_DMA_COPY_SIZE=256"
env $E BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q18_$v$i.json 2>$O/q18_$v$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q18_$v$i.json')); e=[json.loads(l) for l in open('$O/q18_$v$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print('$v', d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)))"
done; done
