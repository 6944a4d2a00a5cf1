set -u
O=gpurun_out; mkdir -p $O
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>&1)"; nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
cat /sys/fs/cgroup/cpu.stat 2>&1 | head -8
for i in 1 2 3; do
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q9_$i.json 2>$O/q9_$i.err || exit 1
python3 -c "
import json; d=json.load(open('$O/q9_$i.json')); e=[json.loads(l) for l in open('$O/q9_$i.err') if l.startswith('{\"sweep')][0]
iv=e['sweep_intervals_ms']; print(d['value'], d['ms_per_step'], max(iv), iv.index(max(iv)))"
cat /sys/fs/cgroup/cpu.stat 2>&1 | grep -E "throttled|usage"
done
