# PMC passes (one counter set per run) over the fp32 eval conv kernels: where do they spend
# their cycles (MFMA busy, VALU, LDS, waits)?  Also lists the gfx950 counters once.
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmc_eval
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_eval/counters.txt 2>&1
SHAPES=${SHAPES:-"f32:eval.layer1 f32:eval.layer2 f32:eval.layer3 f32:eval.layer4 f32:eval.stem"}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/pmc_eval -o p1 -- python3 -m dba_mod_amd.tools.kprobe $SHAPES > $R/gpurun_out/pmc_eval/p1.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_eval -o p2 -- python3 -m dba_mod_amd.tools.kprobe $SHAPES > $R/gpurun_out/pmc_eval/p2.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $R/gpurun_out/pmc_eval -o p3 -- python3 -m dba_mod_amd.tools.kprobe $SHAPES > $R/gpurun_out/pmc_eval/p3.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmc_eval -o kt -- python3 -m dba_mod_amd.tools.kprobe $SHAPES > $R/gpurun_out/pmc_eval/kt.log 2>&1 || exit $?
echo pmc done
