# Round 3: what in a world-1 RCCL group slows the 1-GPU bench: eager vs lazy communicator,
# the init all-reduce, RCCL launch / channel knobs (same box A/B, 12 rounds each).
set -o pipefail
mkdir -p gpurun_out/r3
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps 12 --warmup 2 > gpurun_out/r3/pg9_$tag.log 2>&1 || { tail -20 gpurun_out/r3/pg9_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pg9_$tag.log) $(grep -o '"rccl_ok": [a-z]*' gpurun_out/r3/pg9_$tag.log)"
}
run nopg 29551 X=0
run eager 29552 DBA_FORCE_PG=1
run lazy_nocheck 29553 DBA_FORCE_PG=1 DBA_PG_LAZY=1 DBA_PG_SKIP_SELFCHECK=1
run lazy_check 29554 DBA_FORCE_PG=1 DBA_PG_LAZY=1
run eager_nchan1 29555 DBA_FORCE_PG=1 NCCL_MIN_NCHANNELS=1 NCCL_MAX_NCHANNELS=1
run eager_nomscclpp 29556 DBA_FORCE_PG=1 RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 NCCL_LAUNCH_MODE=GROUP
