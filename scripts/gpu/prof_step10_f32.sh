# rocprofv3 kernel traces of the fp32 training step: 10-client grouped (all active early,
# then the tail) and the lone client (per-kernel latency budget)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for c in ${PROF_CLIENTS:-0 1}; do
  mkdir -p $R/gpurun_out/prof_step$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $R/gpurun_out/prof_step$c/stdout.log 2>&1 || exit $?
done
