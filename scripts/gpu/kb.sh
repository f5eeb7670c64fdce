# microbench fp16 pair + 3 planes, then headline bench
mkdir -p gpurun_out
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --json gpurun_out/kbench_f32_h.json > gpurun_out/kbench_f32_h.log 2>&1 || exit $?
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 3 --reps 10 --json gpurun_out/kbench_f32_p3.json > gpurun_out/kbench_f32_p3.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
