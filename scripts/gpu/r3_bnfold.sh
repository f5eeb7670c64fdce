# Round 3: backward BN finalize folded into the apply (bn_bwd_apply_fin_kernel): bitwise test,
# BN / train-step numerics, lone-step kernel trace, and the step / bench A/B vs three launches.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "bn_bwd_folded or bn_train or train_step_vs_fp64 or solo_tail" > gpurun_out/r3/bnfold_tests.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/r3/bnfold_tests.log | head -20; tail -5 gpurun_out/r3/bnfold_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r3/bnfold_tests.log)"
bash scripts/gpu/prof_step10_f32.sh || exit $?
STEPS=12 bash scripts/gpu/env_ab.sh "X=0" "DBA_BN_BWD_FUSE_G=0" || exit $?
