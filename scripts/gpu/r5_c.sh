# Round 5, call C: where MNIST's round goes (kernel trace of the MNIST bench, per-stream
# tables) and the LOAN / MNIST benches on the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5c
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --config configs/mnist_params.yaml > $O/mnist.log 2>&1 || { tail -20 $O/mnist.log; exit 1; }
echo "mnist: $(grep -o '"value": [0-9.]*' $O/mnist.log) $(grep -o '"phases_mean_s": {[^}]*}' $O/mnist.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/mt -o mnist -- python3 $R/bench.py --config $R/configs/mnist_params.yaml > $O/mnist_prof_stdout.log 2>&1 || { tail -5 $O/mnist_prof_stdout.log; exit 1; }
f=$(find $O/mt -name "*kernel_trace.csv" | head -1)
(cd $R && python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 600 --top 15 > $O/mnist_streams.md) || exit 1
rm -f $f
grep -h '^## stream\|^Window\|^Union' $O/mnist_streams.md
