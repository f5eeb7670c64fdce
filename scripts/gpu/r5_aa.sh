# Round 5, call AA: the poison-phase distances finished on the host (no first-use torch kernels
# in the first poison round): emulated N = 8 rank 0 and the 1-GPU bench (round 203's
# round_ms; state_sha must be unchanged), then the GPU suite and smoke.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5aa
mkdir -p $O
cd $R
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --emulate-rank 0 --emulate-world 8 --round-phases > $O/emu80.log 2>&1 || { tail -20 $O/emu80.log; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --round-phases > $O/n1.log 2>&1 || { tail -20 $O/n1.log; exit 1; }
for f in emu80 n1; do
python3 -c "
import json; j=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', j['value'], j['state_sha'], j['round_ms'][:8])
for e, ph in j['phases_by_round'][:1]: print(e, ph)"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log | cut -c1-200
