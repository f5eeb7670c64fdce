# secondary BASELINE configs at fp32 (1 GPU): RFA, FoolsGold, MNIST, LOAN, Tiny-200
mkdir -p gpurun_out
one() { tag=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/sec_$tag.log 2>&1 || exit $?; echo "$tag: $(tail -1 gpurun_out/sec_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], "acc", d["global_acc"], "asr", d["global_asr"], d["config"]["rounds_timed"])')"; }
one rfa --steps 8 --warmup 2 --aggregation geom_median
one fg --steps 8 --warmup 2 --aggregation foolsgold
one mnist --steps 8 --warmup 2 --config configs/mnist_params.yaml
one loan --steps 8 --warmup 2 --config configs/loan_params.yaml
one tiny200 --steps 6 --warmup 2 --pretrain-rounds 0 --config configs/tiny_200.yaml
