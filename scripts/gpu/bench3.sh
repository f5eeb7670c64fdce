# headline bench three times (run-to-run spread)
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$i.log | cut -c1-140
done
