# Round 5, call X: A/B of the batched model fold (DBA_AB_FOLD) and the fc-weight views
# (DBA_AB_FCVIEW) on one box, interleaved headline benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5x
mkdir -p $O
cd $R
for cfg in 11 00 10 01 11 00; do
f=${cfg:0:1}; v=${cfg:1:1}
DBA_AB_FOLD=$f DBA_AB_FCVIEW=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_$cfg.log 2>&1 || { tail -20 $O/bench_$cfg.log; exit 1; }
python3 -c "import json; j=json.loads(open('$O/bench_$cfg.log').read().strip().splitlines()[-1]); print('bench $cfg', j['value'], j['state_sha'])"
done
