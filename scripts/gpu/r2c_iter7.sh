# register-cached single-launch BN: GPU suite, smoke, lone step, bench, step trace
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log | cut -c1-300
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1.log 2>&1 || exit $?
tail -1 gpurun_out/step1.log | cut -c1-120
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
mkdir -p $R/gpurun_out/prof_step7
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step7 -o step1 -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 1 > $R/gpurun_out/prof_step7/step_stdout.log 2>&1
