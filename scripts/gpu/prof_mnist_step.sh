# step microbenchmark + kernel trace for the MNIST config
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --config configs/mnist_params.yaml --epoch 12 > gpurun_out/mstep.log 2>&1 || exit $?
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --config configs/mnist_params.yaml --epoch 12 --clients 1 >> gpurun_out/mstep.log 2>&1 || exit $?
mkdir -p $R/gpurun_out/mprof
cd /tmp && export TMPDIR=/tmp
PYTHONPATH=$R timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/mprof -o step -- python3 -m dba_mod_amd.tools.bench_step --config $R/configs/mnist_params.yaml --epoch 12 --reps 1 --clients 1 > $R/gpurun_out/mprof/out.log 2>&1
