# PMC counters of the fp16-pair conv kernels (microbench shapes); one pass
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmc_h
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_h -o k -- python3 -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 2 > $R/gpurun_out/pmc_h/stdout.log 2>&1
echo "rc=$?"
ls $R/gpurun_out/pmc_h
