# Round 3: weight gradients on a side stream (models/program.py _wgrad): bitwise / numerics
# tests, then lone / 10-client step and bench A/B (side stream off; finer split-K / wgrad slabs).
set -o pipefail
mkdir -p gpurun_out/r3
DBA_WGRAD_STREAM=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_f32.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "graph_replay or solo_tail or train_step_vs_fp64 or bitwise or two_ranks or warm_model or hip_vs_reference" > gpurun_out/r3/side_tests.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/r3/side_tests.log | head -20; tail -5 gpurun_out/r3/side_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r3/side_tests.log)"
STEPS=12 bash scripts/gpu/env_ab.sh "X=0" "DBA_WGRAD_STREAM=1" "DBA_F32_SPLITK_MINK=4 DBA_F32_SPLITK_TILES=512 DBA_F32_WGRAD_MINROWS=64 DBA_F32_WGRAD_BLOCKS=512" || exit $?
