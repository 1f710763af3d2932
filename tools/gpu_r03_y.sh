# fragment weights + 4-WG logits: batch-1 call profile (greedy and beam 5): per-kernel table of the last call and wall span
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_y; mkdir -p $O
export TMPDIR=/tmp
for beam in 1 5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof$beam -o run -- python3 tools/latency_probe.py 2 $beam > $O/lat_prof$beam.txt 2>&1
  python3 tools/last_call.py $(find $O/prof$beam -name '*kernel_trace.csv' | head -1) > $O/lat_kernels$beam.txt 2>&1
  gzip -f $(find $O/prof$beam -name '*kernel_trace.csv')
done
timeout -k 10 120 python3 tools/latency_probe.py 20 1 > $O/lat1.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "turbo or batch or fused or robust or nan" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for i in 1 2; do timeout -k 10 120 python3 tools/latency_probe.py 30 1 > $O/lat1_$i.txt 2>&1; timeout -k 10 120 python3 tools/latency_probe.py 10 5 > $O/lat5_$i.txt 2>&1; done
grep -h p50 $O/lat*.txt
