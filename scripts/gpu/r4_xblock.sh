# Fused evaluation BasicBlock: its tests, the eval-path tests, then the eval kernel bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_xblock
mkdir -p $O
T=${TESTS:-"tests/test_gpu_xblock.py"}
timeout -k 10 600 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -30
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --only eval --reps 10 > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
grep shape $O/kbench.log
