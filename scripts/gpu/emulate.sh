# Per-rank critical path of an N-rank round, emulated on one GPU (bench.py
# --emulate-rank R --emulate-world N: rank R's clients, early local tests and eval share;
# collectives are counted no-ops).  Every rank of N = 2, 4, 8; ROUNDS timed rounds each
# (default 8: 203..210 holds all four poison rounds; 20: the driver's 203..222 window).
# Extra env (e.g. DBA_EMU_SET="eval_balance=false") is passed through --set.
set -o pipefail
ROUNDS=${ROUNDS:-8}
TAG=${TAG:-emu}
mkdir -p gpurun_out/emu/$TAG
for N in ${WORLDS:-2 4 8}; do
  for R in $(seq 0 $((N - 1))); do
    timeout -k 10 300 python bench.py --emulate-rank $R --emulate-world $N --steps $ROUNDS --warmup ${WARMUP:-2} \
      ${DBA_EMU_SET:+--set $DBA_EMU_SET} > gpurun_out/emu/$TAG/emu_${N}_${R}.log 2>&1 || { tail -20 gpurun_out/emu/$TAG/emu_${N}_${R}.log; exit 1; }
    echo "N=$N R=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/emu/$TAG/emu_${N}_${R}.log) $(grep -o '"train_enqueue": [0-9.]*' gpurun_out/emu/$TAG/emu_${N}_${R}.log) $(grep -o '"eval_wait": [0-9.]*' gpurun_out/emu/$TAG/emu_${N}_${R}.log)"
  done
done
