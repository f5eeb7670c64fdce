# Round 5, call S: the final tree — full GPU suite, smoke, emulated N = 2 / 4 / 8 (every rank, 20 / 5).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5s
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
ROUNDS=20 WARMUP=5 TAG=r5final bash scripts/gpu/r3_emulate.sh
