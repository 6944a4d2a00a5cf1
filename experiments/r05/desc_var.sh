#!/bin/bash
# standalone describe stage times for several libraries
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for L in "$@"; do
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | tail -1 | sed "s|^|$(basename $L .so) |" || exit 1
  DESCRIBE_CFG=5 BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2>/dev/null | tail -1 | sed "s|^|cfg5 $(basename $L .so) |" || exit 1
done
