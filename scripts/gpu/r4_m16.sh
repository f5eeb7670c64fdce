# Same-box A/B of the fused evaluation block's MFMA shape (32x32x16 default build vs the
# XBLOCK_M16=1 build in dba_mod_amd/_lib/ab/): its GPU tests, the block kernel bench, the
# headline bench (driver protocol)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_m16
mkdir -p $O
for v in base M16; do
  if [ $v = base ]; then unset DBA_KERNELS_LIB; else export DBA_KERNELS_LIB=$R/dba_mod_amd/_lib/ab/libdba_kernels_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_xblock.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only "eval.l" > $O/kbench_$v.log 2>&1 || { tail -5 $O/kbench_$v.log; exit 1; }
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only "eval.stem" >> $O/kbench_$v.log 2>&1 || { tail -5 $O/kbench_$v.log; exit 1; }
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "== $v: $(tail -1 $O/tests_$v.log) bench $(grep -o '"value": [0-9.]*' $O/bench_$v.log)"
  grep -h '"eval.layer1"\|"eval.stem"' $O/kbench_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('   ', d['shape'], {k: v for k, v in d.items() if k.endswith('_us')})"
done
