# Round 5, call F: stem weight-gradient kernel (tests, kernel bench, step traces) and the
# synthetic attack-window calibration sweep (r5_e.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5f
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --reps 10 > $O/kbench.log 2>&1 || { tail -20 $O/kbench.log; exit 1; }
grep -E "train\." $O/kbench.log
(cd /tmp && export TMPDIR=/tmp && for c in 1 10; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/step${c}_stdout.log 2>&1 || { tail -5 $O/step${c}_stdout.log; exit 1; }
f=$(find $O/step$c -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.step_trace $f --top 30 > $O/step${c}_trace.md) || exit 1
rm -f $f
head -1 $O/step${c}_trace.md
done) || exit 1
OUT=r5f/sweep bash scripts/gpu/r5_e.sh
