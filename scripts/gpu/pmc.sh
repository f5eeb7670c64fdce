# rocprofv3 hardware counters (MFMA busy, LDS waits / bank conflicts) over the kernel probe
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc -o p1 -- python3 -m dba_mod_amd.tools.kprobe > $R/gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc -o p2 -- python3 -m dba_mod_amd.tools.kprobe > $R/gpurun_out/pmc/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc -o kt -- python3 -m dba_mod_amd.tools.kprobe > $R/gpurun_out/pmc/kt.log 2>&1
