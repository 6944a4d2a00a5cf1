set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_golden.py tests/test_odometry_gpu.py tests/test_edge_gpu.py tests/test_parity_gpu.py tests/test_sequence_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_norm.log 2>&1; rc=$?
tail -3 $O/t_norm.log
[ $rc -eq 0 ] || exit $rc
bash experiments/quick/r03_diag.sh new || exit 1
bash experiments/quick/ab_lib.sh 4
