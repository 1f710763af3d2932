# kernel trace of a short lanes bench (timeline analysis: tools/lane_timeline.py).  usage: gpu_trace.sh OUT [bench args]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline "$@" > $O/bench_prof.json 2> $O/bench_prof.err
gzip -f $O/prof/run_kernel_trace.csv
