# Round 3 perf probes: PMC passes over the fp32 eval convs, then the eval chunk size vs the
# infinity-cache residency of stage-1/2 activations (bench A/B, same box).
set -o pipefail
bash scripts/gpu/pmc_eval.sh || exit $?
mkdir -p gpurun_out/r3
for c in 1024 256 512 1024; do
  timeout -k 10 400 python bench.py --steps 12 --warmup 2 --set eval_batch_size=$c > gpurun_out/r3/bench_chunk$c.log 2>&1 || exit $?
  echo "chunk $c: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3/bench_chunk$c.log)"
done
