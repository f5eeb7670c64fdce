# Round 3: is the RCCL-communicator slowdown GPU-side?  Graph-replayed training steps timed by
# events with and without a live world-1 communicator; then the bench with pairs on/off.
set -o pipefail
mkdir -p gpurun_out/r3
for r in "" "--rccl" ""; do
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 $r > gpurun_out/r3/step_rccl.log 2>&1 || { tail -20 gpurun_out/r3/step_rccl.log; exit 1; }
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 $r > gpurun_out/r3/step1_rccl.log 2>&1 || exit $?
  echo "[$r] step10: $(tail -1 gpurun_out/r3/step_rccl.log | cut -c40-160) | step1: $(tail -1 gpurun_out/r3/step1_rccl.log | cut -c40-100)"
done
