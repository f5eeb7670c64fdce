# small-Cin (stem) kernel: numerics, kernel microbenchmark, 1-GPU bench
mkdir -p gpurun_out/stem
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv_fwd" --timeout 120 --timeout-method thread > gpurun_out/stem/tests.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --only stem > gpurun_out/stem/kbench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/stem/bench.log 2>&1 || exit $?
tail -1 gpurun_out/stem/tests.log; cat gpurun_out/stem/kbench.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/stem/bench.log
