# Round 5, call K: 4-stage operand pipeline of the lone client's 32 x 128 tiles (bitwise tests,
# same-box step A/B), lone-graph prewarm; bench (driver protocol) and the emulated N = 8 ranks.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5k
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_splitk_inlaunch.py tests/test_gpu_bnfuse.py tests/test_gpu_xblock.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for d in 1 0; do
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 3 --deep $d > $O/step1_deep${d}_$i.log 2>&1 || { tail -5 $O/step1_deep${d}_$i.log; exit 1; }
echo "deep=$d rep $i: $(tail -1 $O/step1_deep${d}_$i.log)"
done
done
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 10 --reps 3 > $O/step10.log 2>&1 || { tail -5 $O/step10.log; exit 1; }
echo "10 clients: $(tail -1 $O/step10.log)"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json; j=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print('bench', j['value'], j['round_ms'][:8], j['rounds'][:8])"
for r in 0 1; do
timeout -k 10 300 python bench.py --emulate-rank $r --emulate-world 8 --steps 20 --warmup 5 > $O/emu_8_$r.log 2>&1 || { tail -20 $O/emu_8_$r.log; exit 1; }
python3 -c "import json,sys; j=json.loads(open('$O/emu_8_$r.log').read().strip().splitlines()[-1]); print('emu8 rank $r', j['ms_per_step'], j['round_ms'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step1 -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 2 > $O/step1_stdout.log 2>&1) || { tail -5 $O/step1_stdout.log; exit 1; }
f=$(find $O/step1 -name "*kernel_trace.csv" | head -1)
python3 -m dba_mod_amd.tools.step_trace $f --top 30 > $O/step1_trace.md || exit 1
rm -f $f
head -1 $O/step1_trace.md
