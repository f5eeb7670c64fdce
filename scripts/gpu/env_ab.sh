# Same-box A/B of environment knobs (replaces the round-2 one-off iteration scripts, whose
# knob settings are listed in scripts/gpu/README.md).  Each argument is one configuration,
# a space-separated list of VAR=value ("X=0" = defaults); per configuration: the lone-client
# and 10-client training steps (tools/bench_step) and the 1-GPU headline bench.
#   bash scripts/gpu/env_ab.sh "X=0" "DBA_F32_TRAIN_H_OPS=fwd,dgrad,wgrad"
# STEPS / WARMUP override the bench length (default 20 / 2).
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 1 > gpurun_out/ab/step1_$i.log 2>&1 || { echo "[$cfg] step1 failed"; tail -5 gpurun_out/ab/step1_$i.log; exit 1; }
  env $cfg timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 > gpurun_out/ab/step10_$i.log 2>&1 || { echo "[$cfg] step10 failed"; exit 1; }
  env $cfg timeout -k 10 600 python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-2} > gpurun_out/ab/bench_$i.log 2>&1 || { echo "[$cfg] bench failed"; tail -5 gpurun_out/ab/bench_$i.log; exit 1; }
  echo "[$cfg] step1: $(tail -1 gpurun_out/ab/step1_$i.log | cut -c1-100) | step10: $(tail -1 gpurun_out/ab/step10_$i.log | cut -c1-100) | bench: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/bench_$i.log)"
done
