#!/bin/bash
# round 5 session o: the SHOT gather's 4-byte neighbour indices (keys rebuilt in the rank kernels,
# product build) vs the 8-byte keys (libbshot_base = HEAD 0e1aa6c): GPU suite + smoke, alternating
# bench A/B at configs 1 and 5, a kernel trace and the gather's WRITE_SIZE / FETCH_SIZE per build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05o}
A=b-shot-slam_amd/lib/libbshot_amd.so; B=b-shot-slam_amd/lib/exp/libbshot_base.so
bash scripts/gpu_round.sh $T tests || exit 1
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $A $B | tee $O/${T}_ab_seg32.txt || exit 1
bash experiments/quick/ab_multi.sh 1 $A $B -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_seg32_c5.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for L in $A $B; do
  N=$(basename $L .so)
  BSHOT_LIB=$R/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_$N -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}_$N.json 2> $O/prof_${T}_$N.err || exit 1
  for C in WRITE_SIZE FETCH_SIZE; do
    BSHOT_LIB=$R/$L timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_${T}_${N}_$C -o p --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_${T}_${N}_$C.log 2>&1 || exit 1
  done
done
