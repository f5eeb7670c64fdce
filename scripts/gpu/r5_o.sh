# Round 5, call O: emulated per-rank critical path at N = 2 / 4 / 8 (every rank, the driver's
# 20 / 5 window) on the final tree, and the eval amax-site diagnostic.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd $R
mkdir -p gpurun_out/r5o
timeout -k 10 300 python scripts/diag/eval_amax_sites.py > gpurun_out/r5o/amax_sites.log 2>&1 || { tail -20 gpurun_out/r5o/amax_sites.log; exit 1; }
grep -A30 "amax sites" gpurun_out/r5o/amax_sites.log | head -40
ROUNDS=20 WARMUP=5 TAG=r5emu bash scripts/gpu/r3_emulate.sh
