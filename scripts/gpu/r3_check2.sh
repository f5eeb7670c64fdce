# Round 3: fp32 suite (new stem kernel, near-tie replay gate), e2e additions, smoke under both
# training split policies, RCCL world-1 init, bench A/B of the training-forward split.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_e2e.py -x -v --timeout 300 --timeout-method thread -k "not dba_attack_lands and not hip_vs_reference and not (solo_tail and fp32-mean) and not graph_replay and not gemm3_tile" > gpurun_out/r3/tests2.log 2>&1 || { grep -E "PASSED|FAILED" gpurun_out/r3/tests2.log | tail -5; tail -60 gpurun_out/r3/tests2.log; exit 1; }
tail -1 gpurun_out/r3/tests2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke_default.log 2>&1 || { tail -20 gpurun_out/r3/smoke_default.log; exit 1; }
echo "default: $(tail -1 gpurun_out/r3/smoke_default.log | cut -c1-700)"
DBA_F32_TRAIN_H_OPS=fwd,dgrad,wgrad timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke_hfwd.log 2>&1 || { tail -20 gpurun_out/r3/smoke_hfwd.log; exit 1; }
echo "h-fwd: $(tail -1 gpurun_out/r3/smoke_hfwd.log | cut -c1-700)"
DBA_F32_TRAIN_H_OPS=fwd,dgrad,wgrad timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py -x -v --timeout 300 --timeout-method thread -k "train_step_vs_fp64" > gpurun_out/r3/tests_hfwd.log 2>&1 || { tail -40 gpurun_out/r3/tests_hfwd.log; exit 1; }
tail -1 gpurun_out/r3/tests_hfwd.log
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --dtype fp32 --planes 16 --reps 10 --only stem > gpurun_out/r3/kbench_stem.log 2>&1 || exit $?
cat gpurun_out/r3/kbench_stem.log | grep '^{'
DBA_FORCE_PG=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 \
  > gpurun_out/r3/rccl_world1.log 2>&1 || { tail -30 gpurun_out/r3/rccl_world1.log; exit 1; }
grep '^{' gpurun_out/r3/rccl_world1.log | cut -c1-1200
DBA_F32_TRAIN_H_OPS=fwd,dgrad,wgrad timeout -k 10 400 python bench.py --steps 20 --warmup 2 > gpurun_out/r3/bench_hfwd.log 2>&1 || exit $?
echo "h-fwd bench: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench_hfwd.log) $(grep -o '"rounds": [^]]*]' gpurun_out/r3/bench_hfwd.log | cut -c1-200)"
