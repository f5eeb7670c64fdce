# Round 4 baseline on one box: lone-client and 10-client step kernel traces of the current tree
# (the "before" tables of the training-BN fusion), and the PairAct same-box A/B (20 timed
# rounds after 5 warm-up rounds, DBA_EVAL_PAIRS=1 vs 0, twice each, interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_base
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in 1 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/prof${c}_stdout.log 2>&1 || { echo "trace $c failed"; tail -5 $O/prof${c}_stdout.log; exit 1; }
  f=$(find $O/prof$c -name '*kernel_trace.csv' -print -quit)
  python3 -m dba_mod_amd.tools.step_trace "$f" > $O/step${c}_trace.md || exit 1
  head -1 $O/step${c}_trace.md
done
cd $R
for rep in 1 2; do
  for p in 1 0; do
    DBA_EVAL_PAIRS=$p timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_pairs${p}_$rep.log 2>&1 || { tail -5 $O/bench_pairs${p}_$rep.log; exit 1; }
    echo "pairs=$p rep=$rep $(tail -1 $O/bench_pairs${p}_$rep.log | grep -o '"value": [0-9.]*')"
  done
done
