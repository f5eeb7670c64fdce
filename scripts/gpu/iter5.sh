# fp16 pair in training too (BN-fused operand maxima): numerics, step latency, headline bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -3 gpurun_out/f32_tests.log
[ $rc -eq 0 ] || exit $rc
for m in 3 16; do
  DBA_F32_TRAIN_PLANES=$m timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/step1_m$m.log 2>&1 || exit $?
  DBA_F32_TRAIN_PLANES=$m timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/step10_m$m.log 2>&1 || exit $?
  echo "train planes $m: $(tail -1 gpurun_out/step1_m$m.log | cut -c1-200) | $(tail -1 gpurun_out/step10_m$m.log | cut -c1-200)"
done
DBA_F32_TRAIN_PLANES=16 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h_all.log 2>&1 || exit $?
tail -1 gpurun_out/bench_h_all.log | cut -c1-300
