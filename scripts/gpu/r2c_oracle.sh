# flip-aware oracle: the train-step test with the separate BN pass and with fused BN statistics
for f in 0 1; do
  DBA_BN_FUSED=$f timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -q --timeout 300 --timeout-method thread -k "train_step" > gpurun_out/oracle_$f.log 2>&1
  echo "fused=$f: $(tail -1 gpurun_out/oracle_$f.log)"
  grep -o "AssertionError: ([^)]*)" gpurun_out/oracle_$f.log | head -3
done
