# Persistent LoanNet trainer: its tests, then the LOAN bench (rounds 11..18) with and without it.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_mlp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -10
[ $rc -ne 0 ] && { grep -E "^E " $O/tests.log | head -30; exit $rc; }
[ "${BENCH:-1}" = "0" ] && exit 0
for p in ${MLP_AB:-1 0}; do
  DBA_MLP_PERSIST=$p timeout -k 10 900 python bench.py --config configs/loan_params.yaml > $O/bench_p$p.log 2>&1 || { tail -5 $O/bench_p$p.log; exit 1; }
  echo "persist=$p: $(grep -o "\"value\": [0-9.]*" $O/bench_p$p.log) $(grep -o "\"rounds_timed\": \"[0-9.]*\"" $O/bench_p$p.log) $(grep -o "\"global_acc\": [0-9.]*, \"global_asr\": [0-9.]*" $O/bench_p$p.log)"
done
