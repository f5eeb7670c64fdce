# Round 3: what in a world-1 RCCL group slows the overlapped 1-GPU bench?  Two-stream overlap
# probe (tools/launch_probe) and the bench, each with no group / RCCL communicator / RCCL group
# without a communicator (lazy, no collective) / gloo group.
set -o pipefail
mkdir -p gpurun_out/r3
i=0
for cfg in "X=0" "X=0 --rccl" "DBA_PG_LAZY=1 DBA_PG_SKIP_SELFCHECK=1 --rccl" "X=0 --gloo" "X=0"; do
  i=$((i + 1))
  envs=$(echo $cfg | tr ' ' '\n' | grep '=' | tr '\n' ' '); flags=$(echo $cfg | tr ' ' '\n' | grep -- '--' | tr '\n' ' ')
  env $envs MASTER_PORT=2965$i timeout -k 10 200 python -m dba_mod_amd.tools.launch_probe $flags > gpurun_out/r3/probe$i.log 2>&1 || { tail -20 gpurun_out/r3/probe$i.log; exit 1; }
  echo "probe [$cfg]: $(grep '^{' gpurun_out/r3/probe$i.log)"
done
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps 12 --warmup 2 > gpurun_out/r3/bis_$tag.log 2>&1 || { tail -20 gpurun_out/r3/bis_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bis_$tag.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/bis_$tag.log) $(grep -o '"rccl_ok": [a-z]*' gpurun_out/r3/bis_$tag.log)"
}
run nopg 29661 X=0
run rccl 29662 DBA_FORCE_PG=1
run rccl_nocomm 29663 DBA_FORCE_PG=1 DBA_PG_LAZY=1 DBA_PG_SKIP_SELFCHECK=1
run gloo 29664 DBA_FORCE_PG=1 DBA_DIST_BACKEND=gloo
