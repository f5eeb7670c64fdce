# GPU: kernel unit tests (conv subset) then the conv microbenchmark
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "conv or pconv or sgd" > gpurun_out/t_conv.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/kbench.log
exit $rc
