# The whole GPU tier as the round driver runs it (pytest -m gpu, smoke()), then a short bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_full
mkdir -p $O
T=${TESTS:-tests}
timeout -k 10 1000 python -u -m pytest $T -m gpu -x -v --timeout 600 --timeout-method thread --durations=15 > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -40; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
[ "${BENCH:-1}" = "0" ] && exit 0
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
