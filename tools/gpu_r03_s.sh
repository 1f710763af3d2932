# batcher gap + capture/baton fix: GPU suite, streaming probe (+ kernel trace), config-5 simulation
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_s; mkdir -p $O
export TMPDIR=/tmp


timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/stream_probe.py 3 --sequential-only > $O/stream_probe_prof.txt 2>&1
python3 tools/kstats.py $(find $O/prof -name '*kernel_stats.csv' | head -1) 30 > $O/stream_stats.txt
gzip -f $(find $O/prof -name '*kernel_trace.csv')
timeout -k 10 400 python3 bench.py --steps 1 --warmup 0 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
