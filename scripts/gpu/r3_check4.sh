# Round 3: RCCL host-affinity effect (world-1 group: restored vs kept vs no group) and the
# persistent halo conv with evenly split valid items (bench + grouped step A/B, same box).
set -o pipefail
mkdir -p gpurun_out/r3
rb() {  # $1 label, rest: env assignments; a forced world-1 RCCL group under torchrun
  local tag=$1; shift
  env "$@" DBA_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 > gpurun_out/r3/rccl_$tag.log 2>&1 || { tail -30 gpurun_out/r3/rccl_$tag.log; exit 1; }
  echo "rccl $tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/rccl_$tag.log) $(grep -o '"backend_repinned_cpu_affinity": [a-z]*' gpurun_out/r3/rccl_$tag.log)"
}
rb restored X=0
rb kept DBA_KEEP_RCCL_AFFINITY=1
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/nopg.log 2>&1 || exit $?
echo "no group: $(grep -o '"value": [0-9.]*' gpurun_out/r3/nopg.log)"
for ws in 1 0; do
  DBA_F32_HALO_WS=$ws timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/r3/step10b_ws$ws.log 2>&1 || exit $?
  DBA_F32_HALO_WS=$ws timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench4_ws$ws.log 2>&1 || exit $?
  echo "ws=$ws step10: $(tail -1 gpurun_out/r3/step10b_ws$ws.log | cut -c40-200) bench: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench4_ws$ws.log)"
done
