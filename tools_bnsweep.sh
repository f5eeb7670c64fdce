mkdir -p gpurun_out
for r in 1024 4096 16384; do
  echo "rows=$r" >> gpurun_out/bnsweep.log
  DBA_BN_SMALL_ROWS=$r timeout -k 10 300 python -m dba_mod_amd.tools.bench_step >> gpurun_out/bnsweep.log 2>&1 || exit $?
  DBA_BN_SMALL_ROWS=$r timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --clients 1 >> gpurun_out/bnsweep.log 2>&1 || exit $?
done
