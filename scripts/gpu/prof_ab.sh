# kernel-time A/B of the headline bench (trace, per-stream sums): 8-row halo tiles on / off
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for big in 1 0; do
  mkdir -p $R/gpurun_out/prof_ab$big
  DBA_F32_HALO_BIG=$big timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_ab$big -o bench -- python3 $R/bench.py --steps 6 --warmup 1 --pretrain-rounds 3 > $R/gpurun_out/prof_ab$big/stdout.log 2>&1 || exit $?
  (cd $R && python3 -m dba_mod_amd.tools.trace_streams $(find gpurun_out/prof_ab$big -name "*kernel_trace.csv" | head -1) --last-ms 1500 --top 8 > gpurun_out/prof_ab$big/streams.md)
  echo "big=$big: $(grep -h '^## stream' $R/gpurun_out/prof_ab$big/streams.md | tr '\n' ' ')"
done
