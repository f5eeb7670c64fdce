# 64-wide weight-gradient tiles for small launches: GPU suite, smoke, lone step A/B, bench
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-250
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1.log 2>&1 || exit $?
DBA_F32_WGRAD_BNO64_BLOCKS=0 timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1_b128.log 2>&1 || exit $?
echo "bno64: $(tail -1 gpurun_out/step1.log | cut -c40-110) | bno128: $(tail -1 gpurun_out/step1_b128.log | cut -c40-110)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
