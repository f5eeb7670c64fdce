# Same-box A/B of the xconv register budget (2 workgroups / CU: the default build; 1: the
# dba_mod_amd/_lib/ab/libdba_kernels_minb1.so build): eval + training kernel bench, the lone /
# 10-client step, and the headline bench.
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_minb
mkdir -p $O
for v in 2 1; do
  if [ $v = 1 ]; then export DBA_KERNELS_LIB=$R/dba_mod_amd/_lib/ab/libdba_kernels_minb1.so; else unset DBA_KERNELS_LIB; fi
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 > $O/kbench_$v.log 2>&1 || { tail -5 $O/kbench_$v.log; exit 1; }
  for c in 1 10; do
    timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c > $O/step${c}_$v.log 2>&1 || { tail -5 $O/step${c}_$v.log; exit 1; }
  done
  timeout -k 10 600 python bench.py > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "minb=$v: bench $(grep -o '"value": [0-9.]*' $O/bench_$v.log) step1 $(grep -o '"ms_per_step_by_active": {[^}]*}' $O/step1_$v.log | head -1) step10 $(grep -o '"ms_per_step_by_active": {[^}]*}' $O/step10_$v.log | head -1 | cut -c1-80)"
  grep shape $O/kbench_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('   ', d['shape'], {k: v for k, v in d.items() if k.endswith('_tflops')})"
done
