# Same-box A/B of the headline bench (driver protocol: 20 timed rounds after 5 warm-up rounds):
# $AB_VAR=$v for each v in $AB_VALS (e.g. AB_VAR=DBA_EVAL_BLOCK AB_VALS="1 0").
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/${TAG:-r4_ab}
mkdir -p $O
for v in $AB_VALS; do
  env $AB_VAR=$v timeout -k 10 600 python bench.py > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; exit 1; }
  echo "$AB_VAR=$v: $(grep -o '"value": [0-9.]*' $O/bench_$v.log) $(grep -o '"global_acc": [0-9.]*, "global_asr": [0-9.]*' $O/bench_$v.log)"
done
