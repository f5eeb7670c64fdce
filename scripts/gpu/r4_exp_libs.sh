# Same-box kernel bench of alternative kernel builds (dba_mod_amd/_lib/ab/libdba_kernels_$v.so;
# "base" = the default build): LIBS="base NOSYNC ..." ONLY=<bench_kernels shape filter>
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_exp
mkdir -p $O
for v in ${LIBS:-base}; do
  if [ $v = base ]; then unset DBA_KERNELS_LIB; else export DBA_KERNELS_LIB=$R/dba_mod_amd/_lib/ab/libdba_kernels_$v.so; fi
  timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only "${ONLY:-eval}" > $O/kbench_$v.log 2>&1 || { tail -5 $O/kbench_$v.log; exit 1; }
  echo "== $v"
  grep shape $O/kbench_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('   ', d['shape'], {k: v for k, v in d.items() if k.endswith('_tflops')})"
done
