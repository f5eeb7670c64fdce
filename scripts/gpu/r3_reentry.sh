# Round 3 re-entry: full GPU suite, smoke, headline bench, launch cost with / without a live
# RCCL communicator, bench with a forced world-1 RCCL group (same box).
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3/gpu_tests.log | head; tail -40 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { tail -20 gpurun_out/r3/smoke.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/r3/smoke.log | cut -c1-600)"
timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench.log 2>&1 || { tail -20 gpurun_out/r3/bench.log; exit 1; }
echo "bench: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/bench.log)"
i=0
for r in "" "--rccl" "" "--rccl"; do
  i=$((i + 1))
  MASTER_PORT=2959$i timeout -k 10 200 python -m dba_mod_amd.tools.launch_probe $r > gpurun_out/r3/launch$i.log 2>&1 || { tail -20 gpurun_out/r3/launch$i.log; exit 1; }
  grep '^{' gpurun_out/r3/launch$i.log
done
DBA_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench_pg.log 2>&1 || { tail -20 gpurun_out/r3/bench_pg.log; exit 1; }
echo "bench rccl world-1: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench_pg.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/bench_pg.log)"
