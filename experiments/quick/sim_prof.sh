# kernel trace of the 7-simulated-peer exchange run (replica inserts on the iss stream)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sim7 -o t --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-upload-leg --sim-peers 7 --steps 60 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/prof_sim7.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_sim7.err || exit 1
cd $GRAFT_REPO_ROOT && gzip -c gpurun_out/prof_sim7/t_kernel_trace.csv > gpurun_out/sim7_kernel_trace.csv.gz && rm -rf gpurun_out/prof_sim7/t_kernel_trace.csv && ls gpurun_out/prof_sim7
