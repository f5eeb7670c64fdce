# headline bench at reference precision (fp32, default) and the bf16 fast mode, then a
# rocprofv3 kernel-stats profile of a short fp32 run
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_f32
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_f32.log 2>&1 || exit $?
tail -1 gpurun_out/bench_f32.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --dtype bf16 > gpurun_out/bench_bf16.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bf16.log
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f32 -o bench -- python3 $R/bench.py --steps 4 --warmup 1 --pretrain-rounds 3 > $R/gpurun_out/prof_f32/bench_stdout.log 2>&1
rc=$?; echo "rc=$rc" >> $R/gpurun_out/prof_f32/bench_stdout.log
exit $rc
