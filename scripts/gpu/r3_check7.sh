# Round 3: isolate the world-1 process-group slowdown (same box): no group / RCCL group /
# RCCL with the allocator registration hook off / RCCL with the watchdog monitor off / gloo.
set -o pipefail
mkdir -p gpurun_out/r3
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/pgab_$tag.log 2>&1 || { tail -20 gpurun_out/r3/pgab_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pgab_$tag.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/pgab_$tag.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/pgab_$tag.log) $(grep -o '"train_enqueue": [0-9.]*' gpurun_out/r3/pgab_$tag.log)"
}
run nopg 29531 X=0
run rccl 29532 DBA_FORCE_PG=1
run rccl_nohook 29533 DBA_FORCE_PG=1 TORCH_NCCL_USE_TENSOR_REGISTER_ALLOCATOR_HOOK=0
run rccl_nomon 29534 DBA_FORCE_PG=1 TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0
run gloo 29535 DBA_FORCE_PG=1 DBA_DIST_BACKEND=gloo
