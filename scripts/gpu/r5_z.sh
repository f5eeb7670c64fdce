# Round 5, call Z: kernel timeline of the emulated N = 8 rank 0 (20 / 5): the first poison
# round's slow attacker chain (round_ms 271 vs 88-98 for the later poison rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5z
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5z -o emu -- python3 $R/bench.py --steps 20 --warmup 5 --emulate-rank 0 --emulate-world 8 --round-phases > $O/emu80_prof.log 2>&1) || { tail -5 $O/emu80_prof.log; exit 1; }
f=$(find /tmp/r5z -name "*kernel_trace.csv" | head -1)
python3 -m dba_mod_amd.tools.step_timeline $f --last-ms 1600 > $O/timeline.md
python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 1600 > $O/streams.md
python3 -c "import json; j=json.loads(open('$O/emu80_prof.log').read().strip().splitlines()[-1]); print(j['value'], j['round_ms'][:8])"
head -40 $O/timeline.md
