# A/B of two library builds on one box, alternating: base (experiments/ab/libbshot_base.so, the
# previous commit) vs the tree's lib; default bench line without CPU baseline / upload leg.
# usage: bash experiments/quick/ab_lib.sh <rounds> [bench args]
N=${1:-3}; shift
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then L=experiments/ab/libbshot_base.so; else L=b-shot-slam_amd/lib/libbshot_amd.so; fi
    BENCH_INTERVALS=1 BSHOT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || { tail -5 gpurun_out/ab_$v$i.err; exit 1; }
    python3 -c "
import json
d = json.load(open('gpurun_out/ab_$v$i.json'))
w = [json.loads(l) for l in open('gpurun_out/ab_$v$i.err') if l.startswith('{\"sweep_intervals_ms')][0]['work']
print('$v', $i, d['value'], d['ms_per_step_median'], d['host_ms_per_sweep'], 'work', w)"
  done
done
