#!/bin/bash
# round 5 session q: fills and small copies folded into the ladder build, the SHOT count kernel and
# the map scan (product) vs libbshot_win (HEAD ff02ea9): GPU suite + smoke, alternating bench A/B,
# kernel trace (launches per sweep)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05q}
A=b-shot-slam_amd/lib/libbshot_amd.so; B=b-shot-slam_amd/lib/exp/libbshot_win.so
bash scripts/gpu_round.sh $T tests || exit 1
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $A $B | tee $O/${T}_ab_folds.txt || exit 1
cd /tmp && export TMPDIR=/tmp
BSHOT_LIB=$R/$A timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T} -o trace --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}.json 2> $O/prof_${T}.err
