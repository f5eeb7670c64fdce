# fp32 family: numerics gate, kernel microbench (fp16 pair / 3 bf16 planes), then the headline
# bench with the fp16 pair in evaluation only (training 3 planes) and everywhere
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -3 gpurun_out/f32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --json gpurun_out/kbench_f32_h.json > gpurun_out/kbench_f32_h.log 2>&1 || exit $?
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 3 --reps 10 --json gpurun_out/kbench_f32_p3.json > gpurun_out/kbench_f32_p3.log 2>&1 || exit $?
DBA_F32_PLANES=16 DBA_F32_TRAIN_PLANES=3 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h_eval.log 2>&1 || exit $?
tail -1 gpurun_out/bench_h_eval.log | cut -c1-420
DBA_F32_PLANES=16 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h_all.log 2>&1 || exit $?
tail -1 gpurun_out/bench_h_all.log | cut -c1-420
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_p3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_p3.log | cut -c1-420
