mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t_kernels.log 2>&1 || exit $?
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1 || exit $?
DBA_G3_NS=2 timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench_ns2.json > gpurun_out/kbench_ns2.log 2>&1 || exit $?
timeout -k 10 300 python -m pytest tests/test_gpu_e2e.py -x -q > gpurun_out/t_e2e.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_hip.log 2>&1
