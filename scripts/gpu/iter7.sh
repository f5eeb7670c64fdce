# numerics gate + microbench (fp16 pair) + headline bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -2 gpurun_out/f32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --json gpurun_out/kbench_f32_h.json > gpurun_out/kbench_f32_h.log 2>&1 || exit $?
head -6 gpurun_out/kbench_f32_h.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-250
