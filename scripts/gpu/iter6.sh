# training policy: forward on 3 bf16 planes, gradient passes on the fp16 pair; eval on the pair
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log | cut -c1-600
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/step10.log 2>&1 || exit $?
echo "$(tail -1 gpurun_out/step1.log | cut -c1-120) | $(tail -1 gpurun_out/step10.log | cut -c1-200)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-250
