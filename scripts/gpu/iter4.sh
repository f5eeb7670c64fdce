# fp16-pair iteration: microbench + headline bench with the pair in evaluation
mkdir -p gpurun_out
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --json gpurun_out/kbench_f32_h.json > gpurun_out/kbench_f32_h.log 2>&1 || exit $?
DBA_F32_PLANES=16 DBA_F32_TRAIN_PLANES=3 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h_eval.log 2>&1 || exit $?
tail -1 gpurun_out/bench_h_eval.log | cut -c1-300
