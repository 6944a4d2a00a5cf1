# GPU suite, then (only if green) one default bench line with stage profile; TAG names the outputs
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -2 gpurun_out/pt_$TAG.log
timeout -k 10 200 python bench.py --no-cpu-baseline --profile-stages > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { tail -20 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b_$TAG.json')); print(d['value'], d['upload_inclusive']['value'], d['host_ms_per_sweep'])"
grep -v sweep_int gpurun_out/b_$TAG.err | tail -3
