# PMC passes (one counter set per run, each its own rocprofv3 call) over a probe program:
# MFMA busy / VALU / waits, LDS traffic and conflicts, L2 hits, then a kernel trace.
#   OUT=gpurun_out/pmc PROG="python3 -m dba_mod_amd.tools.kprobe blk stemblk f32:eval.layer2" bash scripts/gpu/pmc.sh
#   PROG="python3 -m dba_mod_amd.tools.bench_step --clients 1 --reps 1"  (the lone-client step)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/${OUT:-gpurun_out/pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P=${PROG:-"python3 -m dba_mod_amd.tools.kprobe blk stemblk f32:eval.layer2"}
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O -o p1 -- $P > $O/p1.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- $P > $O/p2.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d $O -o p3 -- $P > $O/p3.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O -o kt -- $P > $O/kt.log 2>&1 || exit $?
echo pmc done
