# Round 3: which part of the torchrun + RCCL world-1 setup slows the 1-GPU bench (torchrun
# alone / RCCL group alone), then the PMC eval passes and the eval chunk sweep.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 1 --steps 20 --warmup 2 > gpurun_out/r3/torchrun_nopg.log 2>&1 || exit $?
echo "torchrun, no group: $(grep -o '"value": [0-9.]*' gpurun_out/r3/torchrun_nopg.log)"
DBA_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/pg_notorchrun.log 2>&1 || exit $?
echo "RCCL group, no torchrun: $(grep -o '"value": [0-9.]*' gpurun_out/r3/pg_notorchrun.log) $(grep -o '"dist_backend": "[a-z]*"' gpurun_out/r3/pg_notorchrun.log)"
echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"
bash scripts/gpu/r3_perf1.sh || exit $?
