# Round 3: single-launch BN (bn_small_*) for more of the stages: numerics at the larger row
# counts, then lone / 10-client step and bench per threshold (same box).
set -o pipefail
mkdir -p gpurun_out/r3
for r in 4096 16384; do
  DBA_BN_SMALL_ROWS=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bn_train" > gpurun_out/r3/bnsmall_tests_$r.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/r3/bnsmall_tests_$r.log | head -20; exit 1; }
  echo "rows $r tests: $(tail -1 gpurun_out/r3/bnsmall_tests_$r.log)"
done
STEPS=12 bash scripts/gpu/env_ab.sh "X=0" "DBA_BN_SMALL_ROWS=4096" "DBA_BN_SMALL_ROWS=16384"
