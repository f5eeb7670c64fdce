# smoke step vs fp64 in each fp32 split mode, with torch-fp32's own error for reference
mkdir -p gpurun_out
for m in 3 16; do
  DBA_F32_PLANES=$m timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_m$m.log 2>&1; echo "planes $m rc=$?: $(tail -1 gpurun_out/smoke_m$m.log | cut -c1-700)"
done
