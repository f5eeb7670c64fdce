# isolate the Tiny train-step gradient error: fused BN stats / 32-row tiles toggled
T="tests/test_gpu_f32.py::test_fp32_train_step_vs_fp64"
for cfg in "DBA_BN_FUSED=1 DBA_F32_BM32_BLOCKS=256" "DBA_BN_FUSED=0 DBA_F32_BM32_BLOCKS=256" "DBA_BN_FUSED=1 DBA_F32_BM32_BLOCKS=0" "DBA_BN_FUSED=0 DBA_F32_BM32_BLOCKS=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest "$T" -q --timeout 200 --timeout-method thread > gpurun_out/bisect.log 2>&1
  echo "$cfg: $(tail -1 gpurun_out/bisect.log) $(grep -o "AssertionError: ('[a-z0-9_]*', [0-9], [0-9.e-]*" gpurun_out/bisect.log | head -3 | tr '\n' ' ')"
done
