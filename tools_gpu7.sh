mkdir -p gpurun_out
for tpb in 4 8 16 1000000; do
  DBA_PCONV_TPB=$tpb timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_tpb$tpb.log 2>&1 || exit $?
done
DBA_PCONV_TPB=8 timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --json gpurun_out/kbench.json > gpurun_out/kbench.log 2>&1
