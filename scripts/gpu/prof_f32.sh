# rocprofv3 kernel trace + stats of a short fp32 bench run (3 warm-start rounds keep the trace small)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/prof_f32
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f32 -o bench -- python3 $R/bench.py --steps 4 --warmup 1 --pretrain-rounds 3 > $R/gpurun_out/prof_f32/bench_stdout.log 2>&1
rc=$?; echo "rc=$rc" >> $R/gpurun_out/prof_f32/bench_stdout.log
exit $rc
