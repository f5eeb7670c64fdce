# Round 3: per-rank critical path of an N-rank round, emulated on one GPU (bench.py
# --emulate-rank R --emulate-world N: rank R's clients, early local tests and [R::N] test
# shard; collectives are counted no-ops).  Every rank of N = 2, 4, 8; 8 timed rounds each.
set -o pipefail
mkdir -p gpurun_out/r3/emu
timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/r3/emu/world1.log 2>&1 || exit $?
echo "N=1: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3/emu/world1.log)"
for N in 2 4 8; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python bench.py --emulate-rank $R --emulate-world $N --steps 8 --warmup 2 \
      > gpurun_out/r3/emu/emu_${N}_${R}.log 2>&1 || exit $?
    echo "N=$N R=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log) $(grep -o '"train_enqueue": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/r3/emu/emu_${N}_${R}.log)"
  done
done
