# Round 3: BN reduce block size (DBA_BN_BLOCK_ELEMS; fewer rows per block = more blocks for a
# lone client's under-filled BN reduces, more partials for the fused apply to re-sum):
# BN numerics per setting, then the same-box step / bench A/B.
set -o pipefail
export PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/bnblk
for e in 8192 4096; do
  DBA_BN_BLOCK_ELEMS=$e timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bn" > gpurun_out/bnblk/tests_$e.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/bnblk/tests_$e.log | head -20; exit 1; }
  echo "elems $e tests: $(tail -1 gpurun_out/bnblk/tests_$e.log)"
done
STEPS=20 WARMUP=5 bash scripts/gpu/env_ab.sh "X=0" "DBA_BN_BLOCK_ELEMS=8192" "DBA_BN_BLOCK_ELEMS=4096"
