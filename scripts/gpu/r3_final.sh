# Round 3 final-tree check: full GPU suite, smoke, lone-client step kernel trace, 1-GPU bench
# (driver protocol: 20 timed rounds after 5 warm-up rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { grep -E "FAILED|^E " gpurun_out/final/gpu_tests.log | head -30; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/final/prof -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 2 > $R/gpurun_out/final/prof_stdout.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/final/prof_stdout.log; exit 1; }
f=$(find $R/gpurun_out/final/prof -name '*kernel_trace.csv' -print -quit)
python3 -m dba_mod_amd.tools.step_trace "$f" > $R/gpurun_out/final/step1_trace.md || exit 1
head -1 $R/gpurun_out/final/step1_trace.md
cd $R
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/final/step1.log 2>&1 || exit 1
tail -1 gpurun_out/final/step1.log | cut -c1-120
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench.log 2>&1 || { tail -5 gpurun_out/final/bench.log; exit 1; }
tail -1 gpurun_out/final/bench.log | cut -c1-300
