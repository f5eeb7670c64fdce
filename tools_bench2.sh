mkdir -p gpurun_out
timeout -k 10 300 python bench.py --set eval_batch_size=512 > gpurun_out/bench_a.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --set eval_batch_size=512 > gpurun_out/bench_b.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_c.log 2>&1 || exit $?
