# Round 3: which device state does the RCCL communicator init change (limits / flags), and does
# restoring it bring the two-stream overlap back?
set -o pipefail
mkdir -p gpurun_out/r3
i=0
for cfg in "X=0 --rccl" "GPU_MAX_HW_QUEUES=16 --rccl" "X=0 --rccl --same-prio" "X=0 --rccl --streams-first" "X=0 --same-prio" "GPU_MAX_HW_QUEUES=16 --rccl --streams-first"; do
  i=$((i + 1))
  envs=$(echo $cfg | tr ' ' '\n' | grep '=' | tr '\n' ' '); flags=$(echo $cfg | tr ' ' '\n' | grep -- '--' | tr '\n' ' ')
  env $envs MASTER_PORT=2967$i timeout -k 10 200 python -m dba_mod_amd.tools.launch_probe $flags > gpurun_out/r3/lim$i.log 2>&1 || { tail -20 gpurun_out/r3/lim$i.log; exit 1; }
  echo "probe [$cfg]: $(grep '^{' gpurun_out/r3/lim$i.log)"
done
