# Persistent LoanNet trainer: per-step time (tools/bench_mlp) and the LOAN bench's kernel stats.
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_mlp_probe
mkdir -p $O
for g in 1 10; do
  timeout -k 10 120 python -m dba_mod_amd.tools.bench_mlp --G $g --T 400 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o loan -- python3 $R/bench.py --config $R/configs/loan_params.yaml --steps 4 --warmup 1 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
s=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp $s $O/kernel_stats.csv
find $O/prof -name "*kernel_trace.csv" -delete
head -12 $O/kernel_stats.csv | cut -c1-220
