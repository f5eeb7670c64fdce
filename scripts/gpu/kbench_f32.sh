# fp32 family: numerics gate, then per-shape microbenchmarks (3 and 2 split planes)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || exit $?
tail -1 gpurun_out/f32_tests.log
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --planes 3 --reps 10 --json gpurun_out/kbench_f32_p3.json > gpurun_out/kbench_f32_p3.log 2>&1 || exit $?
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --planes 2 --reps 10 --json gpurun_out/kbench_f32_p2.json > gpurun_out/kbench_f32_p2.log 2>&1 || exit $?
cat gpurun_out/kbench_f32_p3.log
