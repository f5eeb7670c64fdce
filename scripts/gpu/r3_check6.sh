# Round 3: does the RCCL group's slowdown come from hardware-queue sharing (GPU_MAX_HW_QUEUES=4
# per process: RCCL's streams + the bench's training / eval streams)?  Same box A/B.
set -o pipefail
mkdir -p gpurun_out/r3
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q DBA_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=2952$q timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/pg_q$q.log 2>&1 || exit $?
  echo "RCCL group, hw queues $q: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pg_q$q.log)"
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/nopg_q$q.log 2>&1 || exit $?
  echo "no group, hw queues $q: $(grep -o '"value": [0-9.]*' gpurun_out/r3/nopg_q$q.log)"
done
