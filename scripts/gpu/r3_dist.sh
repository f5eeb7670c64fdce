# Round 3: RCCL initialisation on a one-GPU box (forced world-1 process group), the default
# 1-GPU headline, and the per-rank emulated critical path for N = 2, 4, 8 (bench.py
# --emulate-rank R --emulate-world N; every rank of every N).
set -o pipefail
mkdir -p gpurun_out/r3
export HSA_ENABLE_IPC_MODE_LEGACY=0
DBA_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 8 --warmup 2 \
  > gpurun_out/r3/rccl_world1.log 2>&1 || exit $?
grep '^{' gpurun_out/r3/rccl_world1.log
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench_default.log 2>&1 || exit $?
grep '^{' gpurun_out/r3/bench_default.log
for N in 2 4 8; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python bench.py --emulate-rank $R --emulate-world $N --steps 8 --warmup 2 \
      > gpurun_out/r3/emu_${N}_${R}.log 2>&1 || exit $?
    echo "N=$N R=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3/emu_${N}_${R}.log)"
  done
done
