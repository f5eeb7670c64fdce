# gen-3 GEMM tile sweep: numerics of every tile code, then the 1-GPU bench per tile choice
# (DBA_G3_SMALL_TILE / DBA_G3_BIG_TILE / DBA_G3_SMALL_LIMIT, codes in ops/hip.py GEMM3_TILES).
# Configs are interleaved and repeated: run-to-run noise of the bench is a few ms.
mkdir -p gpurun_out/g3
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "gemm3_tile or conv_fwd" --timeout 120 --timeout-method thread > gpurun_out/g3/tests.log 2>&1 || exit $?
CFGS=${G3_CFGS:-"0 4 512|2 4 512|6 4 512|2 4 256|0 4 512|2 4 512|6 4 512|2 4 256|1 4 256|2 2 512"}
i=0
IFS='|'
for cfg in $CFGS; do
  IFS=' '
  set -- $cfg
  i=$((i + 1))
  log=gpurun_out/g3/bench_$1_$2_$3_$i.log
  DBA_G3_SMALL_TILE=$1 DBA_G3_BIG_TILE=$2 DBA_G3_SMALL_LIMIT=$3 timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $log)"
  IFS='|'
done
