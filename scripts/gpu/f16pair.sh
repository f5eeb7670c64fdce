# scaled fp16-pair split: numerics gate vs fp64 (all fp32 tests), then microbenchmarks
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -5 gpurun_out/f32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --json gpurun_out/kbench_f32_h.json > gpurun_out/kbench_f32_h.log 2>&1 || exit $?
cat gpurun_out/kbench_f32_h.log
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 3 --reps 10 --json gpurun_out/kbench_f32_p3.json > gpurun_out/kbench_f32_p3.log 2>&1 || exit $?
cat gpurun_out/kbench_f32_p3.log
