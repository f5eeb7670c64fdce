mkdir -p gpurun_out
for eb in 1024 2048 4096; do
  timeout -k 10 300 python bench.py --set eval_batch_size=$eb > gpurun_out/bench_eb$eb.log 2>&1 || exit $?
done
