mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 6 --warmup 2 --set overlap_eval=false > gpurun_out/bench_noovl.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench_noovl.log
exit $rc
