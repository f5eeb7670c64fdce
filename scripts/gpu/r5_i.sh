# Round 5, call I: the calibrated tree's headline bench (driver protocol), its per-stream kernel
# trace (eval-stream kernel ms vs profiles/r4/final3/streams_bench.md), the emulated N = 8
# attacker rank and a benign rank (per-round pacing), and PMC passes over the fused eval blocks.
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5i
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
for r in 0 1; do
timeout -k 10 300 python bench.py --emulate-rank $r --emulate-world 8 --steps 20 --warmup 5 > $O/emu_8_$r.log 2>&1 || { tail -20 $O/emu_8_$r.log; exit 1; }
python3 -c "import json,sys; j=json.loads(open('$O/emu_8_$r.log').read().strip().splitlines()[-1]); print('emu8 rank $r', j['ms_per_step'], j['round_ms'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o bench -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof_stdout.log 2>&1) || { tail -5 $O/prof_stdout.log; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 2000 --top 14 > $O/streams.md || exit 1
rm -f $f
grep -h '^## stream\|^Window\|^Union' $O/streams.md
SHAPES="blk stemblk f32:eval.layer2" bash scripts/gpu/pmc_block.sh
