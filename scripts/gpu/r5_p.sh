# Round 5, call P: the fused block's 4-tile prefetching form — bitwise test, same-box kernel A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5p
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_xblock.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
for t in 1 0; do
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only eval. --tpb $t > $O/kbench_tpb${t}_$i.log 2>&1 || { tail -20 $O/kbench_tpb${t}_$i.log; exit 1; }
echo "tpb=$t rep $i"; grep -E "eval.layer1|chunk" $O/kbench_tpb${t}_$i.log | cut -c1-170
done
done
