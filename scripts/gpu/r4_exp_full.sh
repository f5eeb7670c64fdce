# Same-box A/B of alternative kernel builds (dba_mod_amd/_lib/ab/libdba_kernels_$v.so; "base" =
# the default build): the whole kernel bench and the headline bench per build.  LIBS="base X"
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_expf
mkdir -p $O
for v in ${LIBS:-base}; do
  if [ $v = base ]; then unset DBA_KERNELS_LIB; else export DBA_KERNELS_LIB=$R/dba_mod_amd/_lib/ab/libdba_kernels_$v.so; fi
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only "${ONLY:-}" > $O/kbench_$v.log 2>&1 || { tail -5 $O/kbench_$v.log; exit 1; }
  timeout -k 10 600 python bench.py > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "== $v: bench $(grep -o '"value": [0-9.]*' $O/bench_$v.log)"
  grep shape $O/kbench_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('   ', d['shape'], {k: v for k, v in d.items() if k.endswith('_tflops')})"
done
