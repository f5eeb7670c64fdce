# GPU: all kernel + e2e tests, then bench variants
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -x -q > gpurun_out/t_all.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
for eb in 1024 256 128; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --set eval_batch_size=$eb > gpurun_out/bench_eb$eb.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/bench_eb$eb.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
