# Round 5, call J: XCD-aware block order of the halo convs / fused blocks — bitwise test and a
# same-box kernel A/B on the evaluation shapes (and the training halo rows).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5j
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_xblock.py tests/test_gpu_xdown.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for x in 1 0; do
timeout -k 10 600 python -m dba_mod_amd.tools.bench_kernels --reps 10 --xcd $x > $O/kbench_xcd${x}_$i.log 2>&1 || { tail -20 $O/kbench_xcd${x}_$i.log; exit 1; }
echo "xcd=$x rep $i"; grep -E "eval.layer1|eval.layer2|down|chunk|train.layer1|train.layer2" $O/kbench_xcd${x}_$i.log | cut -c1-170
done
done
