# Round 5, call M: the GPU suite from the e2e file on (call L stopped there), smoke, grouped
# data-gradient in-block slabs (bits + same-box step A/B), headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5m
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_f32.py tests/test_gpu_kernels.py tests/test_gpu_mlp.py tests/test_gpu_splitk_inlaunch.py tests/test_gpu_wgrad.py tests/test_gpu_xblock.py tests/test_gpu_xdown.py tests/test_gpu_ximg.py tests/test_attack_window.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
for i in 1 2; do
for pol in 128,8,8,2,0 128,8,8,2,1 128,8,8,4,1; do
timeout -k 10 300 python -m dba_mod_amd.tools.bench_step --dtype fp32 --clients 10 --reps 3 --split $pol > $O/step10_${pol}_$i.log 2>&1 || { tail -5 $O/step10_${pol}_$i.log; exit 1; }
echo "$pol rep $i: $(tail -1 $O/step10_${pol}_$i.log | cut -c1-260)"
done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
