# lone-step work: fp32 kernel tests, lone / 10-client step (split-K target A/B), bench, step trace
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_step1b
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || { tail -30 gpurun_out/f32_tests.log; exit 1; }
tail -2 gpurun_out/f32_tests.log
for t in 64 128 256; do
  DBA_F32_SPLITK_TILES=$t timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1_t$t.log 2>&1 || exit $?
  DBA_F32_SPLITK_TILES=$t timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/step10_t$t.log 2>&1 || exit $?
  echo "splitk target $t: $(tail -1 gpurun_out/step1_t$t.log | cut -c1-120) | $(tail -1 gpurun_out/step10_t$t.log | cut -c1-200)"
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-300
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step1b -o step1 -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 1 > $R/gpurun_out/prof_step1b/stdout.log 2>&1
