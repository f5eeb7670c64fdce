# PMC passes over the lone-client training step (bench_step --clients 1): the 32 x 128 implicit-GEMM
# tiles of the stage-3/4 convs, the BN passes.  One counter set per run.
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_lone
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 1"
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O -o p1 -- $P > $O/p1.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- $P > $O/p2.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $O -o p3 -- $P > $O/p3.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O -o kt -- $P > $O/kt.log 2>&1 || exit $?
echo pmc done
