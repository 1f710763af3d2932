# GPU tests, then batch-1 latency (greedy and beam 5) with and without one environment
# switch, and a kernel trace of one greedy batch-1 call.  usage: gpu_lat.sh OUT [VAR=VALUE] [pytest -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-lat}; mkdir -p $O
AB=${2:-OSW_NONE=1}
if [ -n "$3" ]; then K=(-k "$3"); else K=(); fi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
for beam in 1 5; do
  timeout -k 10 120 python -u tools/latency_probe.py 20 $beam > $O/lat_a_beam$beam.txt 2>&1
  env $AB timeout -k 10 120 python -u tools/latency_probe.py 20 $beam > $O/lat_b_beam$beam.txt 2>&1
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/latency_probe.py 2 1 > $O/lat_prof.txt 2>&1
python3 tools/last_call.py $O/prof/run_kernel_trace.csv > $O/lat_kernels.txt 2>&1 || true
gzip -f $O/prof/run_kernel_trace.csv
