# Round 5, call AB: idle gaps of the 1-GPU bench's whole timed window (first-use stalls?).
set -o pipefail
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/r5ab
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5ab -o n1 -- python3 $R/bench.py --steps 20 --warmup 5 > $O/n1_prof.log 2>&1) || { tail -5 $O/n1_prof.log; exit 1; }
f=$(find /tmp/r5ab -name "*kernel_trace.csv" | head -1)
python3 -m dba_mod_amd.tools.trace_streams $f --last-ms 6000 > $O/streams_6s.md
grep -A22 "^Idle" $O/streams_6s.md
