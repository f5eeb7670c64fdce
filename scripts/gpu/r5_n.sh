# Round 5, call N: every BASELINE.json config on the final tree with the driver's protocol
# (20 timed rounds after 5 warm-up rounds), one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5n
mkdir -p $O
cd $R
run() {  # tag timeout bench-args...
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  python3 - "$O/$tag.log" "$tag" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], j["value"], j["config"]["rounds_timed"], "acc", j["global_acc"], "asr", j["global_asr"], flush=True)
PY
}
run cifar 600 --steps 20 --warmup 5 || exit 1
run rfa 600 --aggregation geom_median --steps 20 --warmup 5 || exit 1
run fg 600 --aggregation foolsgold --steps 20 --warmup 5 || exit 1
run mnist 300 --config configs/mnist_params.yaml --steps 20 --warmup 5 || exit 1
run loan 600 --config configs/loan_params.yaml --steps 20 --warmup 5 || exit 1
run tiny200 900 --config configs/tiny_200.yaml --pretrain-rounds 0 --steps 20 --warmup 5 || exit 1
