#!/bin/bash
# round 5 session n: the gather's scattered key stores non-temporal (libbshot_ntst) vs plain: bench A/B
# and each build's WRITE_SIZE / FETCH_SIZE per kernel (one counter per pass)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r05n}
bash experiments/quick/ab_multi.sh 2 b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_ntst.so | tee $O/${T}_ab_ntst.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for L in libbshot_amd.so exp/libbshot_ntst.so; do
  N=$(basename $L .so)
  for C in WRITE_SIZE FETCH_SIZE; do
    BSHOT_LIB=$R/b-shot-slam_amd/lib/$L timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_${T}_${N}_$C -o p --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_${T}_${N}_$C.log 2>&1 || exit 1
  done
done
