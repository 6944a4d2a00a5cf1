#!/bin/bash
# round 5: full GPU suite + smoke, alternating bench A/B of library builds, kernel trace of the first
# usage: round_ab.sh <tag> <rounds> <lib>...   (libs relative to the repo root)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=$1; N=$2; shift 2
bash scripts/gpu_round.sh $T tests || exit 1
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh $N "$@" | tee $O/${T}_ab.txt || exit 1
cd /tmp && export TMPDIR=/tmp
BSHOT_LIB=$R/$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T} -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 60 --warmup 10 > $O/prof_${T}.json 2> $O/prof_${T}.err
