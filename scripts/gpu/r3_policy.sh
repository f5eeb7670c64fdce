# Round 3: the communicator queue / priority policy (parallel/dist.py configure_hip_queues) in
# the bench: world-1 RCCL group with the policy vs no group vs the group without it (same box).
set -o pipefail
mkdir -p gpurun_out/r3
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps ${STEPS:-12} --warmup 2 > gpurun_out/r3/pol_$tag.log 2>&1 || { tail -20 gpurun_out/r3/pol_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pol_$tag.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/pol_$tag.log) $(grep -o '"hw_queues": [^,]*, "train_stream_priority": "[-0-9]*"' gpurun_out/r3/pol_$tag.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/pol_$tag.log)"
}
run nopg 29701 X=0
run rccl_policy 29702 DBA_FORCE_PG=1
run rccl_keep 29703 DBA_FORCE_PG=1 DBA_HW_QUEUES=keep
run rccl_policy2 29704 DBA_FORCE_PG=1
run nopg2 29705 X=0
