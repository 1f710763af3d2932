# bench + kernel-trace profile of the same command.  usage: gpu_bench.sh OUT [bench args...]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-bench}; shift || true
mkdir -p $O
timeout -k 10 400 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline --latency-repeats 5 --beam5-latency-repeats 3 --stream-sessions 0 --realistic-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 18 1   # 5+5 greedy + 5+3 beam latency runs
gzip -f $O/prof/run_kernel_trace.csv
