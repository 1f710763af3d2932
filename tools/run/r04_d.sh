# round-4 call 4: per-kernel times of one lane, E-form vs per-head form
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_d; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 3 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ef -o run -- python3 bench.py $A > $O/ef.json 2> $O/ef.err
python3 tools/kstats.py $O/ef/run_kernel_stats.csv 22
OSW_NO_EFORM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ph -o run -- python3 bench.py $A > $O/ph.json 2> $O/ph.err
python3 tools/kstats.py $O/ph/run_kernel_stats.csv 22
rm -f $O/*/run_kernel_trace.csv
