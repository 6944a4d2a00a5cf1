set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
BSHOT_HOST_TRACE=$O/q4_host$i.csv BSHOT_GROW_TRACE=1 BENCH_INTERVALS=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/q4_tr$i -o t --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/q4_drv$i.json 2>$O/q4_drv$i.err || exit 1
python3 -c "import json,sys; d=json.load(open('$O/q4_drv$i.json')); print(d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
