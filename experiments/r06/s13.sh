#!/bin/bash
# round 6 session 13: main-stream kernels that do not fit the LDS SR leaves on a CU (4 KB): k_ham_pair
# with 64-descriptor tiles (3.3 KB instead of 6.5 KB), and SR with a 576-key list (1 KB less per
# workgroup: 16 KB left per CU)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
T=${1:-r06m}
L=b-shot-slam_amd/lib
BSHOT_LIB=$R/$L/ab/libbshot_hk.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "seg_ratio or match or ham" > $O/${T}_pytest_hk.log 2>&1
rc=$?; echo "hk: $(tail -1 $O/${T}_pytest_hk.log)"; [ $rc -eq 0 ] || exit $rc
for V in libbshot_amd ab/libbshot_kc576; do BSHOT_LIB=$R/$L/$V.so timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py | sed "s|^|$V |"; done | tee $O/${T}_sr_bench.txt
rm -f $O/abm_*
BENCH_INTERVALS=1 bash experiments/quick/ab_multi.sh 3 $L/libbshot_amd.so $L/ab/libbshot_hp64.so $L/ab/libbshot_kc576.so $L/ab/libbshot_hk.so | tee $O/${T}_ab.txt || exit 1
for V in amd hp64 kc576 hk; do python experiments/r05/icp_waits.py $O/abm_libbshot_${V}_*.err | grep -v "p75\|p99\|corr"; done > $O/${T}_icp_waits.txt
rm -f $O/abo_*
BENCH_INTERVALS=1 bash experiments/quick/ab_opts.sh 2 sr_run=1 sr_run=2 default | tee $O/${T}_ab_run.txt || exit 1
python experiments/r05/icp_waits.py $O/abo_sr_run_1_*.err $O/abo_sr_run_2_*.err $O/abo_default_*.err | grep -v "p75\|p99\|corr" > $O/${T}_icp_waits_run.txt
