# Round 5, call Q: BN finalize tree tail on wave shuffles (bit-identical: state_sha), BN tests,
# final step traces (lone / 10 clients), headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5q
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnfuse.py tests/test_gpu_splitk_inlaunch.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && for c in 1 10; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/step${c}_stdout.log 2>&1 || { tail -5 $O/step${c}_stdout.log; exit 1; }
f=$(find $O/step$c -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.step_trace $f --top 40 > $O/step${c}_trace.md) || exit 1
rm -f $f
head -1 $O/step${c}_trace.md
grep -E "bnx_finalize|bnx_tile|bnx_dy|amax_seg" $O/step${c}_trace.md
done) || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; j=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print('bench', j['value'], j['state_sha'], j['rounds'][6])"
# Tiny-ImageNet-200: which kernels dominate its round
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tiny -o tiny -- python3 $R/bench.py --config $R/configs/tiny_200.yaml --pretrain-rounds 0 --steps 4 --warmup 1 > $O/tiny_stdout.log 2>&1) || { tail -5 $O/tiny_stdout.log; exit 1; }
s=$(find $O/tiny -name "*kernel_stats.csv" | head -1)
cp $s $O/tiny_kernel_stats.csv
rm -f $(find $O/tiny -name "*kernel_trace.csv")
head -25 $O/tiny_kernel_stats.csv | cut -c1-160
