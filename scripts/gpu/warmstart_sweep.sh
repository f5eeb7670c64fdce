# warm-start lr sweep for Tiny-ImageNet and LOAN (HIP path)
mkdir -p gpurun_out/sweep3
for cfg in "tiny 0.05 40 21" "tiny 0.02 40 21" "loan 0.05 20 10" "loan 0.01 20 10"; do
  set -- $cfg
  d=gpurun_out/sweep3/$1_lr$2_p$3
  mkdir -p $d
  timeout -k 10 300 python main.py --params configs/$1_params.yaml --set resumed_model=false pretrain_rounds=$3 pretrain_lr=$2 start_epoch=$4 max_rounds=8 save_dir=$d > $d/run.log 2>&1 || exit $?
done
