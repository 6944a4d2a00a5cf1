#!/bin/bash
# Counter passes only (no tests): bench line at the driver's size, kernel trace + stats, and the
# FETCH/WRITE and SQ/TCC/GRBM passes of gpu_round.sh, each pass its own run under its own limit.
# usage (via gpurun): bash scripts/pmc_quick.sh <tag>
set -u
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
B="python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2"
echo "[pmc_quick] $(date +%T) bench 20/5" &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err &&
cat $O/bench_driver_$TAG.json &&
cd /tmp && export TMPDIR=/tmp &&
echo "[pmc_quick] $(date +%T) kernel trace" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $O/prof_bench_$TAG.json 2> $O/prof_bench_$TAG.err &&
for P in "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
         "sq1:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
         "sq2:SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR" \
         "tcc:TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
    S=${P%%:*}; C=${P#*:}
    echo "[pmc_quick] $(date +%T) pmc $S"
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc_${S}_$TAG -o $S --output-format csv -- $B > $O/pmc_${S}_$TAG.log 2>&1 || { echo "pass $S failed: $?"; tail -5 $O/pmc_${S}_$TAG.log; exit 1; }
done
echo "[pmc_quick] $(date +%T) done"
