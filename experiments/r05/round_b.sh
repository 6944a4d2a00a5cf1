#!/bin/bash
# round 5 session b: GPU suite + smoke, exchange policy bench, ISS merge A/B (bench + kernel trace)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05b}
bash scripts/gpu_round.sh $T tests || exit 1
bash experiments/r05/xchg.sh $T 2 || exit 1
bash experiments/quick/ab_multi.sh 2 b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_iss32.so || exit 1
cd /tmp && export TMPDIR=/tmp
for L in libbshot_amd.so exp/libbshot_iss32.so; do
  N=$(basename $L .so)
  BSHOT_LIB=$R/b-shot-slam_amd/lib/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_$N -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}_$N.json 2> $O/prof_${T}_$N.err || exit 1
done
