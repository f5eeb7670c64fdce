# In-block split-K slabs for grouped forwards (xconv KS): the bitwise / oracle tests, then the
# 10-client step trace and a same-box headline A/B (DBA_F32_KSLAB=1 default vs 0)
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_kslab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bnfuse.py tests/test_gpu_f32.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for v in ${VALS:-2 0}; do
  DBA_F32_KSLAB=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof10_$v -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 10 --reps 2 > $O/prof10_${v}_stdout.log 2>&1 || { tail -5 $O/prof10_${v}_stdout.log; exit 1; }
  f=$(find $O/prof10_$v -name '*kernel_trace.csv' -print -quit)
  (cd $R && python3 -m dba_mod_amd.tools.step_trace "$f" > $O/step10_trace_$v.md) || exit 1
  rm -f "$f"
  echo "kslab=$v: $(head -1 $O/step10_trace_$v.md)"
done
cd $R
for v in ${VALS:-2 0}; do
  DBA_F32_KSLAB=$v timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "kslab=$v: bench $(grep -o '"value": [0-9.]*' $O/bench_$v.log) $(grep -o '"global_acc": [0-9.]*, "global_asr": [0-9.]*' $O/bench_$v.log)"
done
