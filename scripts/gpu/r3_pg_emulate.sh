# Round 3: world-1 RCCL process-group slowdown A/B (same box, 12 rounds each), then the
# per-rank critical path of N = 2, 4, 8 emulated on one GPU (bench.py --emulate-rank R
# --emulate-world N: rank R's clients, early local tests and eval shard; collectives are
# counted no-ops), every rank, rounds 203..210 (all four poison rounds).
set -o pipefail
mkdir -p gpurun_out/r3/emu
run() {  # $1 tag, $2 port, rest env
  local tag=$1 port=$2; shift 2
  env "$@" MASTER_ADDR=127.0.0.1 MASTER_PORT=$port timeout -k 10 400 python bench.py --steps 12 --warmup 2 > gpurun_out/r3/pgab_$tag.log 2>&1 || { tail -20 gpurun_out/r3/pgab_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pgab_$tag.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/pgab_$tag.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/pgab_$tag.log) $(grep -o '"train_enqueue": [0-9.]*' gpurun_out/r3/pgab_$tag.log)"
}
run nopg 29631 X=0
run pg_streams_first 29632 DBA_FORCE_PG=1
run pg_streams_after 29633 DBA_FORCE_PG=1 DBA_STREAMS_FIRST=0
run pg_q8 29634 DBA_FORCE_PG=1 DBA_STREAMS_FIRST=0 GPU_MAX_HW_QUEUES=8
run pg_ncclhigh 29635 DBA_FORCE_PG=1 DBA_STREAMS_FIRST=0 TORCH_NCCL_HIGH_PRIORITY=1
run nopg2 29636 X=0
for N in 2 4 8; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python bench.py --emulate-rank $R --emulate-world $N --steps 8 --warmup 2 \
      > gpurun_out/r3/emu/emu_${N}_${R}.log 2>&1 || { tail -20 gpurun_out/r3/emu/emu_${N}_${R}.log; exit 1; }
    echo "N=$N R=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log) $(grep -o '"train_enqueue": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log)"
  done
done
