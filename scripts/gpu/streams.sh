# Headline-bench kernel trace: per-stream kernel time over the last 2 s (training stream vs the
# two evaluation streams) and per-kernel totals.  TAG names the output directory.
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
T=${TAG:-streams}
O=$R/gpurun_out/$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o bench -- python3 $R/bench.py --steps 6 --warmup 1 --pretrain-rounds 3 > $O/stdout.log 2>&1 || { tail -5 $O/stdout.log; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 2000 --top 12 > $O/streams.md) || exit 1
s=$(find $O -name "*kernel_stats.csv" | head -1)
[ -n "$s" ] && cp $s $O/kernel_stats.csv
rm -f $f
grep -h '^## stream\|^Window' $O/streams.md
tail -1 $O/stdout.log | cut -c1-200
