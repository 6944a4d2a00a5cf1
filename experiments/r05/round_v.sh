#!/bin/bash
# round 5 session v: k_shot_rank_wg staging with every load in flight (product) vs HEAD 4e6897c
# (libbshot_fold) at config 5, after the describe parity tests; then the ICP list-capacity A/B (round_u.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05v}
L=b-shot-slam_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "describe or rank or hist or config5" > $O/${T}_pytest.log 2>&1
rc=$?; tail -1 $O/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/exp/libbshot_fold.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_rkstage_c5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_c5 -o trace --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload-leg --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 30 --warmup 5 > $O/prof_${T}_c5.json 2> $O/prof_${T}_c5.err || exit 1
cd $R && bash experiments/r05/round_u.sh ${T}u
