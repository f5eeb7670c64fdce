# eval_batch_size sweep of the 1-GPU bench (per-job eval chunk; default 1024)
mkdir -p gpurun_out/sweep
for c in 1024 512 2048 4096 1024; do
  timeout -k 10 300 python bench.py --set eval_batch_size=$c > gpurun_out/sweep/eval_$c.log 2>&1 || exit $?
  echo "chunk $c: $(grep '^{' gpurun_out/sweep/eval_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/sweep/summary.txt
done
