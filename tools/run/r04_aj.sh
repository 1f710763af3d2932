# round-4: batch-1 greedy decode kernel trace (per-step breakdown)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_aj; mkdir -p $O
export TMPDIR=/tmp
set -e
B="--steps 1 --warmup 0 --lanes 1 --latency-repeats 4 --latency-warmup 1 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py $B > $O/b1.json 2> $O/b1.err
python3 tools/b1_breakdown.py $O/prof/run_kernel_trace.csv $((5*445)) > $O/b1_breakdown.txt
rm -f $O/prof/run_kernel_trace.csv
cat $O/b1_breakdown.txt | head -40
