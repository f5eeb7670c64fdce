mkdir -p gpurun_out
DBA_G3_SMALL=1 timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k conv > gpurun_out/t_conv.log 2>&1 || exit $?
DBA_G3_SMALL=1 timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench_small.json > gpurun_out/kbench_small.log 2>&1 || exit $?
DBA_G3_SMALL=1 PYTHONPATH=. timeout -k 10 300 python -m dba_mod_amd.tools.bench_step > gpurun_out/step_small.log 2>&1 || exit $?
PYTHONPATH=. timeout -k 10 300 python -m dba_mod_amd.tools.bench_step > gpurun_out/step.log 2>&1
