# Secondary configs and the headline bench on the current tree (same box)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_cfg
mkdir -p $O
run() {  # $1 tag, $2 timeout, rest bench args
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' $O/$tag.log) $(grep -o '"rounds_timed": "[0-9.]*"' $O/$tag.log) $(grep -o '"global_acc": [0-9.]*, "global_asr": [0-9.]*' $O/$tag.log)"
}
# RUNS: "tag:bench args;tag:bench args;..."
IFS=';' read -ra SPECS <<< "${RUNS:-mnist:--config configs/mnist_params.yaml;cifar:--steps 20 --warmup 5}"
for spec in "${SPECS[@]}"; do
  tag=${spec%%:*}; args=${spec#*:}
  run $tag 600 $args
done
