# fused BN statistics on by default (flip-aware oracle): GPU suite, smoke, steps, bench A/B
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log | cut -c1-300
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/step10.log 2>&1 || exit $?
echo "$(tail -1 gpurun_out/step1.log | cut -c1-110) | $(tail -1 gpurun_out/step10.log | cut -c1-250)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
DBA_BN_FUSED=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nofused.log 2>&1 || exit $?
echo "unfused: $(tail -1 gpurun_out/bench_nofused.log | cut -c1-200)"
