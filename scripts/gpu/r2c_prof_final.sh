# final-tree traces: lone-client step and the headline bench
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_final
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o step1 -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 1 > $R/gpurun_out/prof_final/step_stdout.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o bench -- python3 $R/bench.py --steps 6 --warmup 2 --pretrain-rounds 3 > $R/gpurun_out/prof_final/bench_stdout.log 2>&1
