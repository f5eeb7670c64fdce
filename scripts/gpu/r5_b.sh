# Round 5, call B: fused W-16 downsampling block + fixed-point RFA/FoolsGold sums.
# Targeted GPU tests (incl. world-2 CIFAR bitwise for every aggregation), eval kernel bench,
# same-box bench A/B (DBA_EVAL_DOWN=1 / 0), lone / 10-client training-step traces (baseline).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -x -q --timeout 120 --timeout-method thread > $O/tests_wgrad.log 2>&1 || { tail -30 $O/tests_wgrad.log; exit 1; }
tail -2 $O/tests_wgrad.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_xdown.py tests/test_gpu_kernels.py tests/test_gpu_dist.py tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --reps 10 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -E "down|chunk|train.layer" $O/kbench.log
for i in 1 2; do
for d in 1 0; do
DBA_EVAL_DOWN=$d timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_down${d}_$i.log 2>&1 || { tail -20 $O/bench_down${d}_$i.log; exit 1; }
echo "down=$d rep $i: $(tail -1 $O/bench_down${d}_$i.log | cut -c1-200)"
done
done
cd /tmp && export TMPDIR=/tmp
for c in 1 10; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/step${c}_stdout.log 2>&1 || { tail -5 $O/step${c}_stdout.log; exit 1; }
f=$(find $O/step$c -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.step_trace $f --top 30 > $O/step${c}_trace.md) || exit 1
rm -f $f
head -1 $O/step${c}_trace.md
done
