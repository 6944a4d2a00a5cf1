#!/bin/bash
# SR timing of the `make variant` diagnostic builds (lib/exp/libbshot_<tag>.so) against the default build
# usage: bash scripts/sr_exp.sh [options passed to sr_variants.py, e.g. sr_start=40]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 100 python experiments/sr_variants.py "$@" || exit $?
shopt -s nullglob
for f in b-shot-slam_amd/lib/exp/libbshot_*.so; do
    echo "== $f"
    BSHOT_LIB=$R/$f timeout -k 10 100 python experiments/sr_variants.py "$@" || exit $?
done
