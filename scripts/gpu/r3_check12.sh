# Round 3: eager vs graph-replayed launch sequences with / without a live RCCL communicator,
# then the bench with fp16-pair eval activations on / off (exponent slots without zero-fill).
set -o pipefail
mkdir -p gpurun_out/r3
i=0
for r in "" "--rccl" "" "--rccl"; do
  i=$((i + 1))
  MASTER_PORT=2959$i timeout -k 10 200 python -m dba_mod_amd.tools.launch_probe $r > gpurun_out/r3/launch$i.log 2>&1 || { tail -20 gpurun_out/r3/launch$i.log; exit 1; }
  grep '^{' gpurun_out/r3/launch$i.log
done
for cfg in "DBA_EVAL_PAIRS=0" "DBA_EVAL_PAIRS=1" "DBA_EVAL_PAIRS=0" "DBA_EVAL_PAIRS=1"; do
  env $cfg timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench12.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench12.log)"
done
