# Kernel traces of the isolated roofline and beam-5 passes, as built and with one environment
# switch.  usage: gpu_ab_prof.sh OUT VAR=VALUE
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abp}; mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --latency-repeats 1 --latency-warmup 0 --beam5-latency-repeats 1 --stream-sessions 0 --realistic-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pa -o run -- python3 bench.py $ARGS > $O/bench_a.json 2> $O/bench_a.err
python3 tools/trace_summary.py $O/pa/run_kernel_trace.csv $O/a 2 1
rm -f $O/pa/run_kernel_trace.csv
env $2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pb -o run -- python3 bench.py $ARGS > $O/bench_b.json 2> $O/bench_b.err
python3 tools/trace_summary.py $O/pb/run_kernel_trace.csv $O/b 2 1
rm -f $O/pb/run_kernel_trace.csv
