#!/bin/bash
# One configuration's bench line with its own kernel trace + PMC passes (roofline/limiter from the
# same configuration). usage: bash scripts/gpu_config.sh <tag> <bench args...>
# Output: gpurun_out/summary_<tag>/ (prof_summary.py files + <tag>_bench.json); raw traces dropped.
set -u
TAG=$1; shift
ARGS="$*"
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SHORT="--no-cpu-baseline --no-upload-leg --steps 5 --warmup 2"
echo "[gpu_config] $(date +%T) $TAG kernel trace" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg $ARGS > $O/prof_bench_$TAG.json 2> $O/prof_bench_$TAG.err &&
echo "[gpu_config] $(date +%T) pmc" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o fetch --output-format csv -- \
    python3 $R/bench.py $SHORT $ARGS > $O/pmc_fetch_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o write --output-format csv -- \
    python3 $R/bench.py $SHORT $ARGS > $O/pmc_write_$TAG.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
    -d $O/pmc_sq1_$TAG -o sq1 --output-format csv -- python3 $R/bench.py $SHORT $ARGS > $O/pmc_sq1_$TAG.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR \
    -d $O/pmc_sq2_$TAG -o sq2 --output-format csv -- python3 $R/bench.py $SHORT $ARGS > $O/pmc_sq2_$TAG.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    -d $O/pmc_tcc_$TAG -o tcc --output-format csv -- python3 $R/bench.py $SHORT $ARGS > $O/pmc_tcc_$TAG.log 2>&1 &&
cd $R && python scripts/prof_summary.py $TAG $O/summary_$TAG > /dev/null &&
rm -rf $O/prof_$TAG $O/pmc_fetch_$TAG $O/pmc_write_$TAG $O/pmc_sq1_$TAG $O/pmc_sq2_$TAG $O/pmc_tcc_$TAG &&
echo "[gpu_config] $(date +%T) $TAG bench line" &&
timeout -k 10 900 python bench.py --pmc-file $O/summary_$TAG/${TAG}_pmc.json $ARGS > $O/summary_$TAG/${TAG}_bench.json 2> $O/summary_$TAG/${TAG}_bench.err &&
cat $O/summary_$TAG/${TAG}_bench.json
