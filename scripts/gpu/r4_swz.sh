# ximg LDS swizzle check: its tests, the bank-conflict counters, the kernel bench, the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r4_swz
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ximg.py tests/test_gpu_f32.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^E |FAILED" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O -o p2 -- python3 -m dba_mod_amd.tools.kprobe f32:eval.layer3 f32:eval.layer4 > $O/p2.log 2>&1 || exit $?
cd $R && python3 -m dba_mod_amd.tools.pmc_summary $O --match ximg > $O/summary.md 2>&1; cat $O/summary.md | cut -c1-200
timeout -k 10 300 python -m dba_mod_amd.tools.bench_kernels --reps 10 --only "eval.layer" > $O/kbench.log 2>&1 || { tail -5 $O/kbench.log; exit 1; }
grep shape $O/kbench.log | cut -c1-200
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo "bench $(grep -o '"value": [0-9.]*' $O/bench.log)"
