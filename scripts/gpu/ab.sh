# same-box A/B of the latest evaluation changes
mkdir -p gpurun_out
run() { timeout -k 10 600 env "$@" python bench.py --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || exit $?; echo "$* : $(tail -1 gpurun_out/ab.log | cut -c100-120)"; }
run DBA_EVAL_PAD_C=1 DBA_F32_HALO_BIG=1
run DBA_EVAL_PAD_C=0 DBA_F32_HALO_BIG=1
run DBA_EVAL_PAD_C=1 DBA_F32_HALO_BIG=0
run DBA_EVAL_PAD_C=1 DBA_F32_HALO_BIG=1
