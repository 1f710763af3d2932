# quick GPU check: beam/greedy parity tests + one profiled bench step.  usage: gpu_quick.sh OUT [pytest -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${2:-beam or greedy or sibling}" > $O/gpu_tests.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --latency-repeats 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 1 1
rm -f $O/prof/run_kernel_trace.csv
