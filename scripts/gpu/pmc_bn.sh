# HBM bytes of the training-mode BN kernels (FETCH_SIZE and WRITE_SIZE in separate passes:
# 3 + 2 TCC counters exceed one pass) plus a kernel trace for durations
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
mkdir -p $R/gpurun_out/pmcbn
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmcbn -o fetch -- python3 -m dba_mod_amd.tools.kprobe bn1 bn2 bn3 > $R/gpurun_out/pmcbn/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmcbn -o write -- python3 -m dba_mod_amd.tools.kprobe bn1 bn2 bn3 > $R/gpurun_out/pmcbn/write.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmcbn -o kt -- python3 -m dba_mod_amd.tools.kprobe bn1 bn2 bn3 > $R/gpurun_out/pmcbn/kt.log 2>&1
