# Round 3: kernel traces of the 1-GPU bench without / with a world-1 RCCL group (same box):
# do the kernels run slower under a live communicator, or do the gaps between them grow?
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for tag in nopg rccl; do
  mkdir -p $R/gpurun_out/r3/trace_$tag
  if [ $tag = rccl ]; then export DBA_FORCE_PG=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29641; fi
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3/trace_$tag -o bench -- python3 $R/bench.py --steps 6 --warmup 1 --pretrain-rounds 3 > $R/gpurun_out/r3/trace_$tag/stdout.log 2>&1 || exit $?
  echo "$tag: $(grep -o '"value": [0-9.]*' $R/gpurun_out/r3/trace_$tag/stdout.log)"
done
