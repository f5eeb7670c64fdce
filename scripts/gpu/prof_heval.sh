# kernel trace of the headline bench (fp16 pair in evaluation, 3 planes in training): GPU busy
# fraction vs host enqueue, per-stream kernel time
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/prof_heval
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_heval -o bench -- python3 $R/bench.py --steps 6 --warmup 1 --pretrain-rounds 3 > $R/gpurun_out/prof_heval/bench_stdout.log 2>&1
rc=$?; echo "rc=$rc" >> $R/gpurun_out/prof_heval/bench_stdout.log
[ $rc -eq 0 ] || exit $rc
cd $R && python3 -m dba_mod_amd.tools.trace_streams $(find gpurun_out/prof_heval -name "*kernel_trace.csv" | head -1) --last-ms 1500 --top 14 > gpurun_out/prof_heval/streams.md
tail -3 gpurun_out/prof_heval/streams.md
