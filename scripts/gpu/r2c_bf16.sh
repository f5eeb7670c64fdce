# bf16 fast mode still runs on the current tree (solo tail, register-cached small BN)
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --dtype bf16 > gpurun_out/bench_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bf16.log | cut -c1-300
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype bf16 --clients 1 > gpurun_out/step1_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/step1_bf16.log | cut -c1-120
