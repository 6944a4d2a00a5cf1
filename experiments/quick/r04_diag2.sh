#!/bin/bash
# SR without its ratio computation (diagnostic build) vs product, standalone; config-5 rank kernel A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for L in b-shot-slam_amd/lib/libbshot_amd.so b-shot-slam_amd/lib/exp/libbshot_srnofin.so; do
  BSHOT_LIB=$R/$L timeout -k 10 120 python b-shot-slam_amd/tools/sr_bench.py || exit 1
done
bash experiments/quick/ab_opts.sh 2 default rank_wg=0 -- --sensor 1 --keypoints 4096 --shot-radius 5000 --steps 60 --warmup 10
