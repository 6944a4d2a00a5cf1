cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/pmc_sr1 -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/sr_once.py > $R/gpurun_out/pmc_sr1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES -d $R/gpurun_out/pmc_sr2 -o p --output-format csv -- python3 $R/b-shot-slam_amd/tools/sr_once.py > $R/gpurun_out/pmc_sr2.log 2>&1
