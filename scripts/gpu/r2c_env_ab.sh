# HIP runtime knobs vs the per-launch floor of the lone-client step (graph replay)
for cfg in "X=0" "HIP_FORCE_DEV_KERNARG=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "HIP_FORCE_DEV_KERNARG=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  env $cfg timeout -k 10 200 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 5 > gpurun_out/envab.log 2>&1 || { echo "$cfg failed"; tail -5 gpurun_out/envab.log; exit 1; }
  echo "$cfg: $(tail -1 gpurun_out/envab.log | cut -c40-110)"
done
