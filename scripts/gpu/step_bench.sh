# grouped-step latency (full round and lone attacker), fp32 and bf16, then the headline bench
mkdir -p gpurun_out
for dt in fp32 bf16; do
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype $dt > gpurun_out/step_$dt.log 2>&1 || exit $?
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype $dt --clients 1 > gpurun_out/step1_$dt.log 2>&1 || exit $?
  tail -1 gpurun_out/step_$dt.log; tail -1 gpurun_out/step1_$dt.log
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
