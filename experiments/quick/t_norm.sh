set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "seg_ratio or describe or topk" > $O/t_norm.log 2>&1; rc=$?
tail -3 $O/t_norm.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for L in experiments/ab/libbshot_base.so experiments/ab/libbshot_v1.so b-shot-slam_amd/lib/libbshot_amd.so; do BSHOT_LIB=$(pwd)/$L timeout -k 10 100 python b-shot-slam_amd/tools/sr_bench.py 2>/dev/null | grep lib; done; done
for i in 1 2 3; do for L in experiments/ab/libbshot_base.so experiments/ab/libbshot_v1.so b-shot-slam_amd/lib/libbshot_amd.so; do BSHOT_LIB=$(pwd)/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-upload-leg > $O/b_$i.json 2>/dev/null && python3 -c "import json; d=json.load(open('$O/b_$i.json')); print('$L', d['value'], d['ms_per_step_median'], d['stage_ms_per_sweep'].get('seg_ratio'))"; done; done
