# round-4: batch-1 call kernel times, fused selection vs separate select kernel
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_o; mkdir -p $O
export TMPDIR=/tmp
set -e
B="--steps 1 --warmup 0 --lanes 1 --latency-repeats 3 --latency-warmup 1 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fused -o run -- python3 bench.py $B > $O/fused.json 2> $O/fused.err
python3 tools/kstats.py $O/fused/run_kernel_stats.csv 10
OSW_NO_FUSE_SELECT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sep -o run -- python3 bench.py $B > $O/sep.json 2> $O/sep.err
python3 tools/kstats.py $O/sep/run_kernel_stats.csv 10
rm -f $O/*/run_kernel_trace.csv
python3 -c "import json;print('p50 fused',json.load(open('$O/fused.json'))['p50_latency_ms_b1'],'separate',json.load(open('$O/sep.json'))['p50_latency_ms_b1'])"
