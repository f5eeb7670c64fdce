mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -v --timeout 200 --timeout-method thread -k "train_step or eval_forward" > gpurun_out/arch_tests.log 2>&1 || exit $?
