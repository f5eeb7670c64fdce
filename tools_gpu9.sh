mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_mean.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --aggregation geom_median > gpurun_out/bench_rfa.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --aggregation foolsgold > gpurun_out/bench_fg.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 8 --warmup 2 --config configs/mnist_params.yaml > gpurun_out/bench_mnist.log 2>&1 || exit $?
