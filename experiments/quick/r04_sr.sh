#!/bin/bash
# round 4: SR kernel check -- SR parity tests, standalone SR time (base vs tree), A/B bench, PMC of
# the pipeline's k_seg_ratio (FETCH/WRITE, bank conflicts). usage (gpurun): bash experiments/quick/r04_sr.sh [ab rounds]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
N=${1:-2}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r04_sr_pytest.log 2>&1
rc=$?; tail -3 $O/r04_sr_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base new; do
  if [ $v = base ]; then L=experiments/ab/libbshot_base.so; else L=b-shot-slam_amd/lib/libbshot_amd.so; fi
  BSHOT_LIB=$L timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py || exit 1
done
bash experiments/quick/ab_multi.sh $N experiments/ab/libbshot_base.so b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_hf4.so || exit 1
cd /tmp && export TMPDIR=/tmp
for P in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"; do
  T=$(echo $P | cut -c1-5)
  timeout -s KILL 180 rocprofv3 --pmc $P -d $O/r04pmc_$T -o p --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-upload-leg --steps 5 --warmup 2 > $O/r04pmc_$T.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(o + "/r04pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "k_seg_ratio" in n or "k_hist_fused" in n or "k_lrf" in n:
            agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in agg.items():
    print(n, {k: round(sum(v) / len(v)) for k, v in d.items()})
PY
cd $R
# frame-sharded single sequence, rehearsed with 3 ranks sharing the box's GPU (flow, not scaling)
timeout -k 10 300 python bench.py --gpus 3 --shard-frames --steps 40 --warmup 6 > $O/r04_shard3.json 2> $O/r04_shard3.err && cat $O/r04_shard3.json
