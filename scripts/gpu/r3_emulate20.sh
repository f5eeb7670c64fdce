# Round 3: emulated per-rank critical path over the driver's window (20 timed rounds 203..222,
# warmup 5 as in BENCH_rNN), every rank of N = 2, 4, 8, current defaults; then N = 8 with the
# step latency weighted x4 in the eval balance.
set -o pipefail
ROUNDS=20 WARMUP=5 TAG=emu20 bash scripts/gpu/r3_emulate.sh || exit $?
ROUNDS=20 WARMUP=5 TAG=emu20_lat4800 WORLDS=8 DBA_EMU_SET="balance_step_latency=4800" bash scripts/gpu/r3_emulate.sh || exit $?
