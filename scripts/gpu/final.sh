# Round-end evidence in one call: full GPU suite, smoke, two headline benches, step traces
# (lone / 2-client / 10-client), the stream table of a short bench.  Every GPU step has its own
# time limit and the steps are chained: a failure ends the job.
#   OUT=gpurun_out/<dir> bash scripts/gpu/final.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${OUT:-gpurun_out/final}
mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-400
OUT=${OUT:-gpurun_out/final} N=2 bash scripts/gpu/bench.sh || exit 1
OUT=${OUT:-gpurun_out/final} CLIENTS="1 2 0" bash scripts/gpu/step_trace.sh || exit 1
