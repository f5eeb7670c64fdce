# Round 5, call W: batched fold + split over a flat chunk grid: full GPU
# suite, smoke, the headline bench (state_sha must be unchanged) x2.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5w
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
python3 -c "import json; j=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]); print('bench', j['value'], j['state_sha'])"
done
