# Same-box A/B of fused-BN variants on the lone / 10-client training steps (tools/bench_step
# wall time per step) — each argument one configuration ("X=0" = defaults).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_ab
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > $O/step1_$i.log 2>&1 || { echo "[$cfg] step1 failed"; tail -5 $O/step1_$i.log; exit 1; }
  env $cfg timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > $O/step10_$i.log 2>&1 || { echo "[$cfg] step10 failed"; tail -5 $O/step10_$i.log; exit 1; }
  echo "[$cfg] step1: $(tail -1 $O/step1_$i.log | cut -c1-90) | step10: $(tail -1 $O/step10_$i.log | cut -c1-90)"
done
