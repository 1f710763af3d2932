# batch-1 call profile (greedy and beam 5): per-kernel table of the last call and wall span
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_t; mkdir -p $O
export TMPDIR=/tmp
for beam in 1 5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof$beam -o run -- python3 tools/latency_probe.py 2 $beam > $O/lat_prof$beam.txt 2>&1
  python3 tools/last_call.py $(find $O/prof$beam -name '*kernel_trace.csv' | head -1) > $O/lat_kernels$beam.txt 2>&1
  gzip -f $(find $O/prof$beam -name '*kernel_trace.csv')
done
timeout -k 10 120 python3 tools/latency_probe.py 20 1 > $O/lat1.txt 2>&1
