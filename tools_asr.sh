# synthetic-difficulty sweep of the CIFAR DBA attack window (HIP path)
mkdir -p gpurun_out/sweep2
for cfg in "0.05 0.6 0.5 40" "0.05 0.5 0.5 40" "0.05 0.6 0.4 40" "0.05 0.6 0.5 80" "0.08 0.7 0.5 40"; do
  set -- $cfg
  d=gpurun_out/sweep2/n$1_s$2_c$3_p$4
  mkdir -p $d
  timeout -k 10 200 python main.py --params configs/cifar_params.yaml --set resumed_model=false pretrain_rounds=$4 start_epoch=201 max_rounds=12 synthetic_noise=$1 synthetic_shared=$2 synthetic_clutter=$3 save_dir=$d > $d/run.log 2>&1 || exit $?
done
