# Round 5, call D: MNIST after the two-pass bias gradient and the vectorised max-pool.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5d
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_mlp.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config configs/mnist_params.yaml --steps 20 --warmup 5 > $O/mnist_$i.log 2>&1 || { tail -20 $O/mnist_$i.log; exit 1; }
echo "mnist: $(grep -o '"value": [0-9.]*' $O/mnist_$i.log) $(grep -o '"phases_mean_s": {[^}]*}' $O/mnist_$i.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/mt -o mnist -- python3 $R/bench.py --config $R/configs/mnist_params.yaml > $O/mnist_prof_stdout.log 2>&1 || { tail -5 $O/mnist_prof_stdout.log; exit 1; }
f=$(find $O/mt -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 600 --top 15 > $O/mnist_streams.md) || exit 1
rm -f $f
grep -h '^## stream\|^Window\|^Union' $O/mnist_streams.md
