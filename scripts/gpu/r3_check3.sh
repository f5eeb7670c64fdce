# Round 3: persistent halo conv (correctness + A/B), fp16-pair training forward default,
# stem; kernel microbenchmarks, lone / grouped step, bench A/B (same box), RCCL world-1 effect.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3/tests3.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r3/tests3.log | head; tail -40 gpurun_out/r3/tests3.log; exit 1; }
tail -1 gpurun_out/r3/tests3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke3.log 2>&1 || { tail -20 gpurun_out/r3/smoke3.log; exit 1; }
echo "smoke: $(tail -1 gpurun_out/r3/smoke3.log | cut -c1-400)"
for ws in 1 0; do
  DBA_F32_HALO_WS=$ws timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --only layer1 > gpurun_out/r3/kbench_l1_ws$ws.log 2>&1 || exit $?
  echo "ws=$ws: $(grep '^{' gpurun_out/r3/kbench_l1_ws$ws.log | tr '\n' ' ')"
done
for ws in 1 0; do
  DBA_F32_HALO_WS=$ws timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/r3/step1_ws$ws.log 2>&1 || exit $?
  DBA_F32_HALO_WS=$ws timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/r3/step10_ws$ws.log 2>&1 || exit $?
  echo "ws=$ws step1: $(tail -1 gpurun_out/r3/step1_ws$ws.log | cut -c1-120) | step10: $(tail -1 gpurun_out/r3/step10_ws$ws.log | cut -c1-120)"
done
for cfg in "DBA_F32_HALO_WS=1" "DBA_F32_HALO_WS=0" "DBA_F32_HALO_WS=1"; do
  env $cfg timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench3.log 2>&1 || exit $?
  echo "$cfg: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench3.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/bench3.log)"
  cp gpurun_out/r3/bench3.log gpurun_out/r3/bench3_$(echo $cfg | tr '=' '_').log
done
DBA_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 \
  > gpurun_out/r3/rccl_world1b.log 2>&1 || { tail -30 gpurun_out/r3/rccl_world1b.log; exit 1; }
echo "rccl world-1: $(grep -o '"value": [0-9.]*' gpurun_out/r3/rccl_world1b.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/rccl_world1b.log)"
