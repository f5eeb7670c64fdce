# rocprofv3 kernel trace of the lone-attacker training step (fp32): per-kernel latency budget
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/prof_step
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 2 > $R/gpurun_out/prof_step/stdout.log 2>&1
rc=$?; echo "rc=$rc" >> $R/gpurun_out/prof_step/stdout.log
exit $rc
