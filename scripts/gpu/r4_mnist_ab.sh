# Same-box MNIST A/B of the xconv register budget (default build: 3 workgroups / CU; MINB1 build)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_mnist_ab
mkdir -p $O
for v in base MINB1 base; do
  if [ $v = base ]; then unset DBA_KERNELS_LIB; else export DBA_KERNELS_LIB=$R/dba_mod_amd/_lib/ab/libdba_kernels_$v.so; fi
  timeout -k 10 300 python bench.py --config configs/mnist_params.yaml > $O/mnist_$v.log 2>&1 || { tail -5 $O/mnist_$v.log; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' $O/mnist_$v.log) $(grep -o '"phases_mean_s": {[^}]*}' $O/mnist_$v.log)"
done
