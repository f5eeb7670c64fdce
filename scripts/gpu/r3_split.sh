# Round 3: where a 1-GPU round goes — training and evaluation serialised (overlap_eval=false:
# phases "train" vs "eval_wait"), the overlapped default, and the grouped / lone training step.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python bench.py --steps 12 --warmup 2 --set overlap_eval=false > gpurun_out/r3/bench_serial.log 2>&1 || { tail -20 gpurun_out/r3/bench_serial.log; exit 1; }
echo "serial: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench_serial.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/bench_serial.log)"
timeout -k 10 400 python bench.py --steps 12 --warmup 2 > gpurun_out/r3/bench_overlap.log 2>&1 || { tail -20 gpurun_out/r3/bench_overlap.log; exit 1; }
echo "overlap: $(grep -o '"value": [0-9.]*' gpurun_out/r3/bench_overlap.log) $(grep -o '"phases_mean_s": {[^}]*}' gpurun_out/r3/bench_overlap.log)"
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/r3/step10.log 2>&1 || { tail -20 gpurun_out/r3/step10.log; exit 1; }
echo "step10: $(tail -1 gpurun_out/r3/step10.log)"
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/r3/step1.log 2>&1 || { tail -20 gpurun_out/r3/step1.log; exit 1; }
echo "step1: $(tail -1 gpurun_out/r3/step1.log)"
