#!/bin/bash
# standalone describe stage times: product vs diagnostic k_hist_fused builds (no apply / no records)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O; cd $R
for L in b-shot-slam_amd/lib/libbshot_amd.so ${EXTRA_LIBS:-}; do
  echo "== $L"
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py || exit 1
done
