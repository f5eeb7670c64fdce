# kernel + e2e GPU tests, then the step microbenchmark and a 1-GPU bench
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step > gpurun_out/step.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --clients 1 >> gpurun_out/step.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
