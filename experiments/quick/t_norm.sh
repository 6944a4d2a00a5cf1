set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_norm.log 2>&1; rc=$?
tail -3 $O/t_norm.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do for L in experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so; do BSHOT_LIB=$(pwd)/$L timeout -k 10 100 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | grep total; done; done
bash experiments/quick/ab_lib.sh 3
