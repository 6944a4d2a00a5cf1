#!/bin/bash
# host timeline (BSHOT_HOST_TRACE) + kernel trace of a short bench run, for pipeline analysis
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-th}
cd /tmp && export TMPDIR=/tmp
export BSHOT_HOST_TRACE=$R/gpurun_out/${TAG}_host.csv
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/$TAG -o t --output-format csv -- \
    python3 $R/bench.py --no-cpu-baseline --steps 12 --warmup 3 ${@:2} > $R/gpurun_out/$TAG.log 2>&1
