# Round 3: fp16-pair evaluation activations — numerics (fp32 suite + e2e eval tests + smoke),
# eval kernel microbenchmarks, and the bench A/B (same box).
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 120 --timeout-method thread -k "eval_pair" > gpurun_out/r3/tests_pairs.log 2>&1 || { grep -E "PASSED|FAILED" gpurun_out/r3/tests_pairs.log; grep -E "^E " gpurun_out/r3/tests_pairs.log | head -20; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/r3/tests_pairs.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke10.log 2>&1 || { tail -20 gpurun_out/r3/smoke10.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/r3/smoke10.log | cut -c1-500)"
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --only eval > gpurun_out/r3/kbench_eval10.log 2>&1 || exit $?
grep '^{' gpurun_out/r3/kbench_eval10.log
for cfg in "DBA_EVAL_PAIRS=1" "DBA_EVAL_PAIRS=0" "DBA_EVAL_PAIRS=1"; do
  env $cfg timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench10.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench10.log) $(grep -o '"global_acc": [0-9.]*' gpurun_out/r3/bench10.log)"
  cp gpurun_out/r3/bench10.log gpurun_out/r3/bench10_$(echo $cfg | tr '=' '_').log
done
