set -u
for q in 4 8 4 8 4 8; do
echo -n "HWQ=$q "; GPU_MAX_HW_QUEUES=$q bash scripts/exp_bench.sh "" || exit 1
done
for q in 4 8; do
GPU_MAX_HW_QUEUES=$q BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/q15_d$q.json 2>gpurun_out/q15_d$q.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/q15_d$q.json')); print('driver HWQ=$q', d['value'], d['ms_per_step'])"
done
