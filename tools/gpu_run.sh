set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r13}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 5 1
gzip -f $O/prof/run_kernel_trace.csv
ls -la $O/prof
