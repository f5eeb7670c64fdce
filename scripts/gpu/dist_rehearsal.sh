# 2 ranks sharing the one GPU of the box, gloo collectives: rehearses the multi-rank round
# pipeline (placement, early/sharded eval, gather, aggregation) on real HIP kernels
mkdir -p gpurun_out
DBA_SHARE_GPU=1 DBA_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 > gpurun_out/rehearsal.log 2>&1
