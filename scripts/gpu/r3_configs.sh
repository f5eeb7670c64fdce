# Round 3: secondary BASELINE configs on the final tree (RFA / FoolsGold CIFAR, Tiny, MNIST,
# LOAN) and Tiny-ImageNet-200 over all four of its poison rounds (21..28).
set -o pipefail
mkdir -p gpurun_out/r3
run() {  # $1 tag, $2 timeout, rest bench args
  local tag=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > gpurun_out/r3/cfg_$tag.log 2>&1 || { tail -20 gpurun_out/r3/cfg_$tag.log; exit 1; }
  echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3/cfg_$tag.log) $(grep -o '"rounds_timed": "[0-9.]*"' gpurun_out/r3/cfg_$tag.log) $(grep -o '"global_acc": [0-9.]*, "global_asr": [0-9.]*' gpurun_out/r3/cfg_$tag.log)"
}
run rfa 400 --aggregation geom_median
run fg 400 --aggregation foolsgold
run mnist 300 --config configs/mnist_params.yaml
run loan 300 --config configs/loan_params.yaml
run tiny200 1000 --config configs/tiny_200.yaml --pretrain-rounds 0 --steps 8 --warmup 2
