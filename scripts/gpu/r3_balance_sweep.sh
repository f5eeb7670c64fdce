# Round 3: eval-balance cost model sweep on the emulated per-rank critical path (same box):
# even strided split vs water-filling with the default / doubled step-latency weight.
set -o pipefail
for cfg in "even eval_balance=false" "lat1200 balance_step_latency=1200" "lat2400 balance_step_latency=2400"; do
  tag=${cfg%% *}; set_=${cfg#* }
  TAG=sweep_$tag WORLDS="${WORLDS:-2 8}" DBA_EMU_SET="$set_" bash scripts/gpu/r3_emulate.sh || exit $?
done
