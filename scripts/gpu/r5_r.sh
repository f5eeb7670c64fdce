# Round 5, call R: the XCD remap removed (it confined a sparsely active grouped step to 1-2 XCDs),
# the vector weight gradient for Wo 2 / 1 (Tiny stage 4); tests, step traces, CIFAR + Tiny benches
# (state_sha unchanged = same bits).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5r
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_xblock.py tests/test_gpu_wgrad.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
(cd /tmp && export TMPDIR=/tmp && for c in 1 10; do
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/step$c -o step -- python3 -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 2 > $O/step${c}_stdout.log 2>&1 || { tail -5 $O/step${c}_stdout.log; exit 1; }
f=$(find $O/step$c -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.step_trace $f --top 40 > $O/step${c}_trace.md) || exit 1
rm -f $f
head -1 $O/step${c}_trace.md
done) || exit 1
for cfg in "cifar:--steps 20 --warmup 5" "tiny200:--config configs/tiny_200.yaml --pretrain-rounds 0 --steps 20 --warmup 5"; do
tag=${cfg%%:*}; args=${cfg#*:}
timeout -k 10 900 python bench.py $args > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
python3 -c "import json; j=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1]); print('$tag', j['value'], j['state_sha'])"
done
