# fp32 (reference-precision) kernel family: numerics vs fp64, determinism, train step
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || exit $?
