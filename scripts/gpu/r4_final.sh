# End-of-round check of the final tree: the GPU tier as the driver runs it (pytest -m gpu,
# smoke, bench), the fused-BN tests + lone / 10-client step traces + the driver-protocol bench
# (r4_bnx.sh), then MFMA-utilisation counters of the evaluation convs (one pass per counter set)
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu/r4_full.sh || exit $?
TESTS="tests/test_gpu_bnfuse.py" bash $R/scripts/gpu/r4_bnx.sh || exit $?
export PYTHONPATH=$R
O=$R/gpurun_out/r4_final_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
S="f32:eval.layer1 f32:eval.layer2 f32:eval.layer3 f32:eval.layer4"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O -o p1 -- python3 -m dba_mod_amd.tools.kprobe $S > $O/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- python3 -m dba_mod_amd.tools.kprobe $S > $O/p2.log 2>&1 || exit $?
cd $R && python3 -m dba_mod_amd.tools.pmc_summary $O > $O/summary.md 2>&1 || true
echo final done
