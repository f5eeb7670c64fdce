# PMC counters of the persistent LoanNet trainer (tools/bench_mlp, 10 clients x 400 steps)
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_mlp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d $O -o p1 -- python3 -m dba_mod_amd.tools.bench_mlp --G 10 --T 400 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH --output-format csv -d $O -o p2 -- python3 -m dba_mod_amd.tools.bench_mlp --G 10 --T 400 > $O/p2.log 2>&1 || exit 1
cd $R && for f in $(find $O -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if "mlp_train" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1].split("/")[-1], {k: round(v) for k, v in sorted(agg.items())})
PY
done
