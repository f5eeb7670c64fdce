# Attack-window calibration sweep: the bench window (8 timed rounds 203..210 after 5 warm-up)
# under synthetic-data / knob settings, one line of round:acc/ASR per setting.
#   OUT=gpurun_out/calib CFGS="X=0|--set synthetic_sky=0.12|DBA_FUSED_HEAD=0" bash scripts/gpu/calib.sh
# (each configuration: environment assignments and/or bench.py arguments; "X=0" = defaults)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/${OUT:-gpurun_out/calib}
mkdir -p $O
cd $R
i=0
IFS='|' read -ra CS <<< "${CFGS:-X=0}"
for cfg in "${CS[@]}"; do
  i=$((i + 1))
  envs=""; args=""
  for tok in $cfg; do
    case "$tok" in
      [A-Z_]*=*) envs="$envs $tok" ;;
      *) args="$args $tok" ;;
    esac
  done
  env $envs timeout -k 10 400 python bench.py --steps ${STEPS:-8} --warmup 5 $args > $O/calib_$i.log 2>&1 || { tail -20 $O/calib_$i.log; exit 1; }
  python3 -c "
import json; j=json.loads(open('$O/calib_$i.log').read().strip().splitlines()[-1])
print('[$cfg]', ' '.join(f'{r}:{a:.0f}/{s:.0f}' for r, a, s in j['rounds']), j['value'], j.get('state_sha'))"
done
