#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench line, rocprofv3 kernel stats, HBM PMC passes.
# Every GPU step has its own time limit and the chain stops at the first failure.
# usage (from the repo root, via gpurun): bash scripts/gpu_round.sh [tag] [all|tests|perf]
# (tests and perf as two gpurun calls keep each under gpurun's 20-minute limit)
set -u
TAG=${1:-r01}
PART=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ "$PART" != perf ]; then
echo "[gpu_round] $(date +%T) pytest -m gpu" &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1 &&
tail -3 $O/pytest_gpu_$TAG.log &&
echo "[gpu_round] $(date +%T) smoke" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 &&
cat $O/smoke_$TAG.log || exit 1
fi
[ "$PART" = tests ] && exit 0
echo "[gpu_round] $(date +%T) bench" &&
timeout -k 10 600 python bench.py --profile-stages > $O/bench_$TAG.json 2> $O/bench_$TAG.err &&
cat $O/bench_$TAG.json &&
echo "[gpu_round] $(date +%T) bench, driver-sized (20 steps, 5 warm-up)" &&
BENCH_INTERVALS=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err &&
cat $O/bench_driver_$TAG.json &&
echo "[gpu_round] $(date +%T) host timeline (no profiler)" &&
BSHOT_HOST_TRACE=$O/host_$TAG.csv timeout -k 10 300 python bench.py --no-cpu-baseline --no-upload-leg --steps 100 --warmup 10 > $O/bench_host_$TAG.json 2>&1 &&
python b-shot-slam_amd/tools/host_phases.py $O/host_$TAG.csv > $O/host_phases_$TAG.txt &&
cat $O/host_phases_$TAG.txt &&
cd /tmp && export TMPDIR=/tmp &&
echo "[gpu_round] $(date +%T) rocprofv3 kernel trace" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG -o trace --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline > $O/prof_bench_$TAG.json 2> $O/prof_bench_$TAG.err &&
echo "[gpu_round] $(date +%T) pmc FETCH_SIZE" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$TAG -o fetch --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_fetch_$TAG.log 2>&1 &&
echo "[gpu_round] $(date +%T) pmc WRITE_SIZE" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$TAG -o write --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_write_$TAG.log 2>&1 &&
echo "[gpu_round] $(date +%T) pmc SQ pass 1" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
    -d $O/pmc_sq1_$TAG -o sq1 --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_sq1_$TAG.log 2>&1 &&
echo "[gpu_round] $(date +%T) pmc SQ pass 2" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR \
    -d $O/pmc_sq2_$TAG -o sq2 --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_sq2_$TAG.log 2>&1 &&
echo "[gpu_round] $(date +%T) pmc TCC/TCP/GRBM pass" &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    -d $O/pmc_tcc_$TAG -o tcc --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/pmc_tcc_$TAG.log 2>&1 &&
echo "[gpu_round] $(date +%T) preprocessor + capture kernels" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pre_$TAG -o t --output-format csv -- \
    python3 $R/b-shot-slam_amd/tools/pre_bench.py 30 > $O/pre_bench_$TAG.log 2>&1 &&
grep "^{" $O/pre_bench_$TAG.log > $O/pre_bench_$TAG.json &&
cat $O/pre_bench_$TAG.json &&
echo "[gpu_round] $(date +%T) summaries -> gpurun_out/summary_$TAG (raw traces dropped, kernel trace gzipped)" &&
cd $R && python scripts/prof_summary.py $TAG $O/summary_$TAG &&
gzip -c $O/prof_$TAG/trace_kernel_trace.csv > $O/summary_$TAG/${TAG}_kernel_trace.csv.gz &&
rm -rf $O/prof_$TAG $O/pmc_fetch_$TAG $O/pmc_write_$TAG $O/pmc_sq1_$TAG $O/pmc_sq2_$TAG $O/pmc_tcc_$TAG $O/prof_pre_$TAG &&
du -sh $O &&
echo "[gpu_round] $(date +%T) done"
