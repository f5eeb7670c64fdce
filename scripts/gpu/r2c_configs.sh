# secondary configs on the current tree + a kernel trace of the headline bench
R=$GRAFT_REPO_ROOT
bash scripts/gpu/bench_all_configs.sh || exit $?
for f in rfa fg tiny mnist loan; do echo "$f: $(tail -1 gpurun_out/bench_$f.log | cut -c1-160)"; done
bash scripts/gpu/bench_tiny200.sh > gpurun_out/tiny200_stdout.log 2>&1 || exit $?
tail -1 gpurun_out/tiny200_stdout.log | cut -c1-200
mkdir -p $R/gpurun_out/prof_bench6
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench6 -o bench -- python3 $R/bench.py --steps 6 --warmup 2 --pretrain-rounds 3 > $R/gpurun_out/prof_bench6/stdout.log 2>&1
