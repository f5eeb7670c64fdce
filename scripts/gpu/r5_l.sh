# Round 5, call L: the full GPU suite and smoke on the current tree, step traces, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5l
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
(cd /tmp && export TMPDIR=/tmp && for c in 1 10; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/step${c}_stdout.log 2>&1 || { tail -5 $O/step${c}_stdout.log; exit 1; }
f=$(find $O/step$c -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.step_trace $f --top 40 > $O/step${c}_trace.md) || exit 1
rm -f $f
head -1 $O/step${c}_trace.md
done) || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
