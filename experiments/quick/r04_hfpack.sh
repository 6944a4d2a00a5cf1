#!/bin/bash
# packed SHOT apply: LDS lane-order microbench, describe parity with the packed builds, standalone
# describe times (product, packed, diagnostics), then a bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 60 ./experiments/microbench/lds_lane_order || exit 1
for L in hfp12 hfp8; do
  BSHOT_LIB=$R/b-shot-slam_amd/lib/exp/libbshot_$L.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "describe or golden or shot or config5" > $O/r04_${L}_pytest.log 2>&1
  rc=$?; echo "$L: $(tail -1 $O/r04_${L}_pytest.log)"; [ $rc -eq 0 ] || { tail -30 $O/r04_${L}_pytest.log; exit $rc; }
done
EXTRA_LIBS="b-shot-slam_amd/lib/exp/libbshot_hfp8.so b-shot-slam_amd/lib/exp/libbshot_hfp12.so b-shot-slam_amd/lib/exp/libbshot_hfd1.so b-shot-slam_amd/lib/exp/libbshot_hfd2.so" bash experiments/quick/r04_hfdiag.sh || exit 1
bash experiments/quick/ab_multi.sh ${1:-2} b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_hfp12.so b-shot-slam_amd/lib/exp/libbshot_hfp8.so
