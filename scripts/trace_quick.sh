#!/bin/bash
# kernel + memory-copy timeline of a short bench run (no counters)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tq}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/$TAG -o t --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 2 > $R/gpurun_out/$TAG.log 2>&1
