# Round 5, call H: split-K policy sweep of the training step (lone client = the N = 8 attacker's
# chain; 10 clients = the 1-GPU round): target tiles, min k-steps per slab, max slabs, max in-block slabs.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
for pol in ${POLS:-128,8,8,2 256,4,8,2 256,4,8,4 256,4,8,8 512,4,8,8 256,8,8,4}; do
  for c in 1 10; do
    timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients $c --reps 3 --split $pol > $O/step${c}_$pol.log 2>&1 || { tail -5 $O/step${c}_$pol.log; exit 1; }
    echo "$pol clients=$c $(tail -1 $O/step${c}_$pol.log)"
  done
done
