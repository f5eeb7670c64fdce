# last-block BN finalize: fp32 / e2e / dist suites, steps, bench, launch-knob A/B, step trace
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_e2e.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32e2e_tests.log 2>&1 || { tail -40 gpurun_out/f32e2e_tests.log; exit 1; }
tail -2 gpurun_out/f32e2e_tests.log
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1.log 2>&1 || exit $?
DBA_BN_LAST_BLOCK=0 timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1_nolb.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/step10.log 2>&1 || exit $?
echo "$(tail -1 gpurun_out/step1.log | cut -c1-110) | no-lb $(tail -1 gpurun_out/step1_nolb.log | cut -c40-110) | $(tail -1 gpurun_out/step10.log | cut -c1-250)"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
bash scripts/gpu/r2c_env_ab.sh || exit $?
mkdir -p $R/gpurun_out/prof_step5
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step5 -o step1 -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 1 > $R/gpurun_out/prof_step5/step_stdout.log 2>&1
