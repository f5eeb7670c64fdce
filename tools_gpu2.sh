mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t_kernels.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_kernels.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_e2e.py -x -q > gpurun_out/t_e2e.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_e2e.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_hip.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench_hip.log
exit $rc
