# Round 3: at N > 1, local tests on the owner rank right after training (early_local_eval) vs
# every test image-sharded by the water-filling split (emulated per-rank critical path).
set -o pipefail
TAG=early_off WORLDS="${WORLDS:-2 8}" DBA_EMU_SET="early_local_eval=false" bash scripts/gpu/r3_emulate.sh || exit $?
