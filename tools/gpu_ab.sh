# quick GPU check + A/B of one environment switch.  usage: gpu_ab.sh OUT "pytest -k expr" VAR=VALUE
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > $O/gpu_tests.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --latency-repeats 3 --beam5-steps 0 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 3 1
rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 240 python -u bench.py --steps 6 --beam5-steps 0 --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err
env $3 timeout -k 10 240 python -u bench.py --steps 6 --beam5-steps 0 --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err
