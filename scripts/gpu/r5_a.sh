# Round 5, first call: the pruned fp16-pair-only tree + the fused downsampling block.
# GPU tier (every test), smoke, kernel microbenchmarks (eval shapes, fused vs two-launch
# downsampling block, whole 17x1024 eval chunk), the driver-protocol bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --only eval --reps 10 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
cat $O/kbench.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
DBA_EVAL_DOWN=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_down0.log 2>&1 || { tail -20 $O/bench_down0.log; exit 1; }
tail -1 $O/bench_down0.log | cut -c1-400
