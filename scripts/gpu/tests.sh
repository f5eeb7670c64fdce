# GPU tests (a subset with TESTS="tests/test_x.py ..."), one process, per-test timeout
#   OUT=gpurun_out/<dir> TESTS="tests/test_gpu_bnfuse.py" bash scripts/gpu/tests.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${OUT:-gpurun_out/tests}
mkdir -p $O
cd $R
timeout -k 10 ${TLIMIT:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
exit $rc
