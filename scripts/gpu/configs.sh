# secondary BASELINE configs on one MI355X: RFA / FoolsGold defenses (CIFAR), Tiny-ImageNet, MNIST, LOAN
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --aggregation geom_median > gpurun_out/bench_rfa.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --aggregation foolsgold > gpurun_out/bench_fg.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config configs/tiny_params.yaml --steps 6 > gpurun_out/bench_tiny.log 2>&1 || exit $?
timeout -k 10 1000 python bench.py --config configs/tiny_200.yaml --steps 20 --warmup 5 > gpurun_out/bench_tiny200.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config configs/mnist_params.yaml > gpurun_out/bench_mnist.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config configs/loan_params.yaml > gpurun_out/bench_loan.log 2>&1 || exit $?
