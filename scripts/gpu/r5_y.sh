# Round 5, call Y: per-round host phases of the first poison round (N = 8 emulated rank 0 and
# N = 1): where round 203's extra ~35 ms goes.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5y
mkdir -p $O
cd $R
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --emulate-rank 0 --emulate-world 8 --round-phases > $O/emu80.log 2>&1 || { tail -20 $O/emu80.log; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --round-phases > $O/n1.log 2>&1 || { tail -20 $O/n1.log; exit 1; }
for f in emu80 n1; do
python3 -c "
import json; j=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', j['value'], j['round_ms'][:8])
for e, ph in j['phases_by_round'][:8]: print(e, ph)"
done
