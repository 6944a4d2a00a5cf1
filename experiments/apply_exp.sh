#!/bin/bash
# standalone describe stage times (tools/describe_bench.py) for the default build and every
# `make variant` build under lib/exp (e.g. HA_G / HA_LDS_PAD of k_hist_apply); bits/SHOT hashes
# must agree across builds
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2 || exit $?
shopt -s nullglob
for f in b-shot-slam_amd/lib/exp/libbshot_*.so; do
    echo "== $f"
    BSHOT_LIB=$R/$f timeout -k 10 120 python b-shot-slam_amd/tools/describe_bench.py 2 || exit $?
done
