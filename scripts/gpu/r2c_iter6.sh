# solo tail (a lone client's last steps in the G=1 graph): GPU suite, smoke, bench A/B
R=$GRAFT_REPO_ROOT
export DBA_SOLO_MIN_STEPS=4
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log | cut -c1-300
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
DBA_SOLO_MIN_STEPS=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_nosolo.log 2>&1 || exit $?
echo "no solo: $(tail -1 gpurun_out/bench_nosolo.log | cut -c1-200)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench2.log 2>&1 || exit $?
echo "solo again: $(tail -1 gpurun_out/bench2.log | cut -c1-200)"
