# rocprofv3 kernel traces of the fp32 training step for 1, 2 and all (10) clients of a poison
# round, summarised per step by tools/step_trace (kernels/step, us/step, per-kernel table).
#   OUT=gpurun_out/<dir> CLIENTS="1 2 0" bash scripts/gpu/step_trace.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/${OUT:-gpurun_out/steps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CLIENTS:-1 2 0}; do
  rm -rf /tmp/st$c
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/st$c -o step -- python3 -m dba_mod_amd.tools.bench_step --clients $c --reps 3 > $O/bench_step$c.log 2>&1 || { tail -20 $O/bench_step$c.log; exit 1; }
  f=$(find /tmp/st$c -name "*kernel_trace.csv" | head -1)
  python3 -m dba_mod_amd.tools.step_trace $f --top 40 > $O/step${c}_trace.md || exit 1
  tail -1 $O/bench_step$c.log
  head -1 $O/step${c}_trace.md
done
