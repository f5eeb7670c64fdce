mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --config configs/mnist_params.yaml --epoch 12 > gpurun_out/mstep.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config configs/mnist_params.yaml > gpurun_out/bench_mnist.log 2>&1 || exit $?
