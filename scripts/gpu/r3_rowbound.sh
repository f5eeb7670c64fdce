# Round 3: coalesced multi-block row_bound (PairAct output bound at eval fold): tests, bench,
# kernel stats of a short bench.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -k "row_bound or eval_pair or eval_forward or warm_model or fl_rounds or bitwise" > gpurun_out/r3/rb_tests.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/r3/rb_tests.log | head -20; tail -5 gpurun_out/r3/rb_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r3/rb_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/rb_smoke.log 2>&1 || { tail -20 gpurun_out/r3/rb_smoke.log; exit 1; }
for i in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r3/rb_bench$i.log 2>&1 || { tail -20 gpurun_out/r3/rb_bench$i.log; exit 1; }
  echo "bench $i: $(grep -o '"value": [0-9.]*' gpurun_out/r3/rb_bench$i.log)"
done
bash scripts/gpu/prof_bench.sh || exit $?
