# GPU: all tests, kernel microbench, bench
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -x -q > gpurun_out/t_all.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/kbench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_hip.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench_hip.log
exit $rc
