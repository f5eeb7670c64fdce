# kernel statistics of the lone-client training step: 3 bf16 planes vs the fp16 pair
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in 3 16; do
  DBA_F32_TRAIN_PLANES=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step_m$m -o run -- python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 --reps 2 > gpurun_out/prof_step_m$m.log 2>&1 || exit $?
done
find gpurun_out/prof_step_m3 gpurun_out/prof_step_m16 -name "*kernel_stats.csv" | head
