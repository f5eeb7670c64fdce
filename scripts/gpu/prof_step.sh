# grouped-step microbenchmark (all clients / one client) + kernel trace
mkdir -p gpurun_out
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step > gpurun_out/step.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --clients 1 >> gpurun_out/step.log 2>&1 || exit $?
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/profstep
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profstep -o step -- python3 -m dba_mod_amd.tools.bench_step --reps 1 --clients 1 > $R/gpurun_out/profstep/out.log 2>&1
