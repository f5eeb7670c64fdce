# smoke step error vs fp64 with the fp16 pair on one conv pass at a time
mkdir -p gpurun_out
for ops in fwd dgrad wgrad; do
  DBA_F32_PLANES=16 DBA_F32_H_OPS=$ops timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$ops.log 2>&1; echo "$ops rc=$?: $(tail -1 gpurun_out/smoke_$ops.log | grep -o "'grad_rel_err.*eval_logits_rel_err': [0-9.e-]*")"
done
