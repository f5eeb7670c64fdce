# Round 3: in-launch split-K combine (xgemm.hip sk_combine) — bitwise tests vs the separate
# reduce launch, the full GPU suite, lone-step kernel traces with the combine on / off, and a
# same-box step / bench A/B (DBA_F32_SK_INLAUNCH=0 = the separate xsplitk_reduce launches).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
export DBA_SK_COUNTERS=${DBA_SK_COUNTERS:-32768}   # training steps take the in-launch combine
mkdir -p gpurun_out/sk
timeout -k 10 300 python -u -m pytest tests/test_gpu_splitk_inlaunch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sk/tests_new.log 2>&1 || { tail -40 gpurun_out/sk/tests_new.log; exit 1; }
tail -1 gpurun_out/sk/tests_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sk/gpu_tests.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/sk/gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/sk/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sk/smoke.log 2>&1 || { tail -5 gpurun_out/sk/smoke.log; exit 1; }
tail -1 gpurun_out/sk/smoke.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  DBA_F32_SK_INLAUNCH=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/sk/prof$v -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 2 > $R/gpurun_out/sk/prof_stdout_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $R/gpurun_out/sk/prof_stdout_$v.log; exit 1; }
  f=$(find $R/gpurun_out/sk/prof$v -name '*kernel_trace.csv' -print -quit)
  python3 -m dba_mod_amd.tools.step_trace "$f" > $R/gpurun_out/sk/step1_trace_$v.md || exit 1
  head -1 $R/gpurun_out/sk/step1_trace_$v.md
done
cd $R
STEPS=20 WARMUP=5 bash scripts/gpu/env_ab.sh "X=0" "DBA_F32_SK_INLAUNCH=0"
