# Round 3 check: smoke (near-tie replay), the new / changed GPU tests, RCCL world-1 init, bench
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { tail -20 gpurun_out/r3/smoke.log; exit 1; }
tail -1 gpurun_out/r3/smoke.log | cut -c1-900
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_f32.py -x -v --timeout 300 --timeout-method thread -k "graph_replay or solo_tail or warm_model or train_step_vs_fp64" > gpurun_out/r3/tests1.log 2>&1 || { tail -40 gpurun_out/r3/tests1.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r3/tests1.log | tail -20
DBA_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 8 --warmup 2 \
  > gpurun_out/r3/rccl_world1.log 2>&1 || { tail -30 gpurun_out/r3/rccl_world1.log; exit 1; }
grep '^{' gpurun_out/r3/rccl_world1.log | cut -c1-1500
