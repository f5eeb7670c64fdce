# 1-GPU headline bench on the driver protocol (20 timed rounds after 5 warm-up), N times:
#   OUT=gpurun_out/<dir> N=2 ARGS="--set aggregation_methods=foolsgold" bash scripts/gpu/bench.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${OUT:-gpurun_out/bench}
mkdir -p $O
cd $R
for i in $(seq 1 ${N:-1}); do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 $ARGS > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  python3 -c "import json; j=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]); print('bench', j['value'], j.get('state_sha'), [round(x) for x in j.get('round_ms', [])])"
done
