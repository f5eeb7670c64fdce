# eval_max_groups sweep of the 1-GPU bench (jobs per grouped eval launch; default 24)
mkdir -p gpurun_out/gsweep
for g in 24 8 48 24; do
  timeout -k 10 300 python bench.py --set eval_max_groups=$g > gpurun_out/gsweep/g_$g.log 2>&1 || exit $?
  echo "groups $g: $(grep '^{' gpurun_out/gsweep/g_$g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/gsweep/summary.txt
done
