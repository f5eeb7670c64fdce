# Round 3: training-stream priority and hardware-queue count under a live RCCL communicator
# (the communicator breaks the overlap of a high-priority stream with a default-priority one:
# profiles/rccl_probe_r3.jsonl).  Bench A/B on one box.
set -o pipefail
mkdir -p gpurun_out/r3
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps 12 --warmup 2 > gpurun_out/r3/prio_$tag.log 2>&1 || { tail -20 gpurun_out/r3/prio_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/prio_$tag.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/prio_$tag.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/prio_$tag.log)"
}
run nopg_hi 29691 X=0
run nopg_hi_q8 29692 GPU_MAX_HW_QUEUES=8
run nopg_same_q8 29693 DBA_TRAIN_STREAM_PRIORITY=0 GPU_MAX_HW_QUEUES=8
run rccl_hi_q8 29694 DBA_FORCE_PG=1 GPU_MAX_HW_QUEUES=8
run rccl_same_q8 29695 DBA_FORCE_PG=1 DBA_TRAIN_STREAM_PRIORITY=0 GPU_MAX_HW_QUEUES=8
run rccl_same_q6 29696 DBA_FORCE_PG=1 DBA_TRAIN_STREAM_PRIORITY=0 GPU_MAX_HW_QUEUES=6
run nopg_hi2 29697 X=0
