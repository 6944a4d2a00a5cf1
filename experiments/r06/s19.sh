#!/bin/bash
# round 6 session 19: describe gather staged in LDS (segments <= 8192 entries, product) vs the direct
# scatter (sg0) vs 16384-entry staging (sg16k): parity, per-kernel write bytes (config 2 and 5),
# standalone describe, alternating benches at config 2 and config 5
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06t}
L=b-shot-slam_amd/lib
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_odometry_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or shot or golden or config5" > $O/${T}_pytest.log 2>&1
rc=$?; echo "product: $(tail -1 $O/${T}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
BSHOT_LIB=$R/$L/ab/libbshot_sg16k.so timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "describe or shot" > $O/${T}_pytest_sg16k.log 2>&1
rc=$?; echo "sg16k: $(tail -1 $O/${T}_pytest_sg16k.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_sg0 ab/libbshot_sg16k libbshot_amd ab/libbshot_sg0 ab/libbshot_sg16k; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | sed "s|^|$V |" || exit 1; done | tee $O/${T}_describe_bench.txt
cd /tmp && export TMPDIR=/tmp
for V in libbshot_amd ab/libbshot_sg0 ab/libbshot_sg16k; do
  for C in c2 c5; do
    A="--no-cpu-baseline --no-upload-leg --steps 5 --warmup 2"; [ $C = c5 ] && A="$A --sensor 1 --keypoints 4096 --shot-radius 5000"
    N=$(basename $V); rm -rf $O/w_${T}_${N}_$C
    BSHOT_LIB=$R/$L/$V.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/w_${T}_${N}_$C -o w --output-format csv -- python3 $R/bench.py $A > $O/w_${T}_${N}_$C.log 2>&1 || { echo "pmc $N $C failed"; exit 1; }
    echo "$N $C"; python3 $R/experiments/r06/wsize.py $(find $O/w_${T}_${N}_$C -name "w_counter_collection.csv" | head -1)
    rm -rf $O/w_${T}_${N}_$C
  done
done | tee $O/${T}_write_bytes.txt
cd $R
rm -f $O/abm_*
bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_sg0.so $L/ab/libbshot_sg16k.so | tee $O/${T}_ab.txt || exit 1
bash experiments/quick/ab_multi.sh 2 $L/libbshot_amd.so $L/ab/libbshot_sg0.so $L/ab/libbshot_sg16k.so -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10 | tee $O/${T}_ab_c5.txt || exit 1
