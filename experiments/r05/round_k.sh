#!/bin/bash
# round 5 session k: exchange + ICP tests on HEAD, map-insert sort with 512 threads vs 1024 (config 2 and 5)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05k}
timeout -k 10 600 python -u -m pytest tests/test_xchg_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "xchg or exchange or icp or replica" > $O/${T}_pytest.log 2>&1
rc=$?; tail -2 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash experiments/quick/ab_multi.sh 2 b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_sort512.so | tee $O/${T}_ab_sort_c2.txt || exit 1
bash experiments/quick/ab_multi.sh 1 b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_sort512.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_sort_c5.txt
