# BASELINE config #3: Tiny-ImageNet ResNet-18, 200 Dirichlet clients, DBA, fp32 (central warm start)
mkdir -p gpurun_out
timeout -k 10 1000 python bench.py --config configs/tiny_200.yaml --pretrain-rounds 0 --steps 6 --warmup 2 > gpurun_out/bench_tiny200.log 2>&1 || exit $?
tail -1 gpurun_out/bench_tiny200.log
