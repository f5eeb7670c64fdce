# Fused training BN bring-up: its unit tests, the whole-step oracle / replay / solo-tail tests,
# then (only if they pass) lone / 10-client step traces and a short bench.
# TESTS overrides the pytest selection; TRACE=0 stops after the tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_bnx
mkdir -p $O
T=${TESTS:-"tests/test_gpu_bnfuse.py tests/test_gpu_f32.py::test_fp32_train_step_vs_fp64 tests/test_gpu_e2e.py::test_train_step_hip_vs_reference tests/test_gpu_e2e.py::test_graph_replay_matches_eager tests/test_gpu_e2e.py::test_solo_tail_bitwise"}
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40
[ $rc -ne 0 ] && { grep -E "^E |Error|error" $O/tests.log | head -40; exit $rc; }
[ "${TRACE:-1}" = "0" ] && exit 0
cd /tmp && export TMPDIR=/tmp
for c in 1 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/prof${c}_stdout.log 2>&1 || { echo "trace $c failed"; tail -5 $O/prof${c}_stdout.log; exit 1; }
  f=$(find $O/prof$c -name '*kernel_trace.csv' -print -quit)
  python3 -m dba_mod_amd.tools.step_trace "$f" > $O/step${c}_trace.md || exit 1
  head -1 $O/step${c}_trace.md
done
cd $R
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
