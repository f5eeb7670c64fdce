# Synthetic attack-window calibration sweep (verdict r4 item 7): per-round global clean acc /
# global-trigger ASR over the CIFAR window 203..210 and the MNIST window 12..19 (driver protocol:
# 5 warm-up rounds) for generator settings given as "name|config|--set overrides" lines in
# $SETS (default: the list below).  One bench run per setting, each under its own limit.
set -o pipefail
out=gpurun_out/${OUT:-r5e}
mkdir -p $out
run() {  # name config overrides...
  local name=$1 cfg=$2; shift 2
  timeout -k 10 240 python bench.py --config configs/$cfg --steps 8 --warmup ${WARMUP:-5} --set "$@" \
    > $out/$name.log 2> $out/$name.err || return $?
  python - "$out/$name.log" "$name" >> $out/summary.txt <<'EOF'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], " ".join(f"{r}:{a:.0f}/{s:.0f}" for r, a, s in j["rounds"]), j["value"], flush=True)
EOF
}
SETS=${SETS:-"c_sky0|cifar_params.yaml|synthetic_sky=0
c_sky30|cifar_params.yaml|synthetic_sky=0.3
c_sky45|cifar_params.yaml|synthetic_sky=0.45
c_sky30_n07|cifar_params.yaml|synthetic_sky=0.3 synthetic_noise=0.07 synthetic_shared=0.65
m_m0|mnist_params.yaml|synthetic_margin=0
m_m4|mnist_params.yaml|synthetic_margin=4
m_m4_s5|mnist_params.yaml|synthetic_margin=4 synthetic_shared=0.5"}
while IFS='|' read -r name cfg sets; do
  [ -z "$name" ] && continue
  run $name $cfg $sets || exit $?
done <<< "$SETS"
cat $out/summary.txt
