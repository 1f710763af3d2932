# kernel profile of the isolated greedy and beam-5 passes of the current tree
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --latency-repeats 3 --beam5-latency-repeats 0 --beam5 1 --beam5-steps 0 --stream-sessions 0 --realistic-steps 0 > $O/bench.json 2> $O/bench.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 3 1
rm -f $O/prof/run_kernel_trace.csv
head -14 $O/s_beam5_pass.txt
