# fused BN statistics with NaN-poisoned partial buffers: does any slot stay unwritten?
export DBA_BN_FUSED=1 DBA_BN_FUSED_POISON=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -q --timeout 300 --timeout-method thread -k "train_step or bn_stats_folded" > gpurun_out/poison.log 2>&1
tail -15 gpurun_out/poison.log | grep -v "^$"
grep -o "AssertionError: ([^)]*)" gpurun_out/poison.log | head
