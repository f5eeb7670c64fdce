# Round 5, call T: implicit-GEMM tile rows (automatic / 64 / 128) on every kernel-bench shape.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5t
mkdir -p $O
cd $R
for i in 1 2; do
for bm in 0 64 128; do
timeout -k 10 400 python -m dba_mod_amd.tools.bench_kernels --reps 10 --bm $bm > $O/kbench_bm${bm}_$i.log 2>&1 || { tail -20 $O/kbench_bm${bm}_$i.log; exit 1; }
echo "bm=$bm rep $i done"
done
done
