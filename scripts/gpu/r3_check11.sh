# Round 3: is the RCCL-communicator slowdown GPU-side?  Graph-replayed training steps timed by
# events with and without a live world-1 communicator (interleaved, distinct logs).
set -o pipefail
mkdir -p gpurun_out/r3
i=0
for r in "" "--rccl" "" "--rccl"; do
  i=$((i + 1))
  MASTER_PORT=2957$i timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 $r > gpurun_out/r3/step10_rccl$i.log 2>&1 || { tail -20 gpurun_out/r3/step10_rccl$i.log; exit 1; }
  MASTER_PORT=2958$i timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 $r > gpurun_out/r3/step1_rccl$i.log 2>&1 || exit $?
  echo "[$r] step10: $(grep -o '"ms_per_step_by_active": {[^}]*}' gpurun_out/r3/step10_rccl$i.log) | step1: $(grep -o '"ms_per_step_by_active": {[^}]*}' gpurun_out/r3/step1_rccl$i.log)"
done
