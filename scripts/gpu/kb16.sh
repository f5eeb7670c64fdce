# halo W16 A/B (fp16 pair microbench), numerics first
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1; rc=$?
tail -1 gpurun_out/f32_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  DBA_F32_HALO16=$v timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --only layer2 > gpurun_out/kb16_$v.log 2>&1 || exit $?
  echo "halo16=$v"; grep -v amdgpu gpurun_out/kb16_$v.log | cut -c1-200
done
