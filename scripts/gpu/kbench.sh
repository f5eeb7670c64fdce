# fp32 family: numerics gate (SKIP_TESTS=1 skips it), then the per-shape kernel microbenchmarks
#   OUT=gpurun_out/kbench ONLY=eval bash scripts/gpu/kbench.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${OUT:-gpurun_out/kbench}
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > $O/f32_tests.log 2>&1 || { tail -20 $O/f32_tests.log; exit 1; }
  tail -1 $O/f32_tests.log
fi
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --reps ${REPS:-10} ${ONLY:+--only $ONLY} --json $O/kbench.json > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log
