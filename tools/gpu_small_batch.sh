# Small-batch encoder profile (config 2 / config 5): kernel stats of log-mel + encoder +
# cross-K/V at 1 and 4 windows, then the streaming call probe.  usage: gpu_small_batch.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
for B in 1 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$B -o run -- python3 tools/encoder_run.py --batch $B --iters 10 > $O/b$B.log 2>&1
  python3 tools/kstats.py $(find $O/b$B -name '*kernel_stats.csv' | head -1) 30 > $O/b${B}_stats.txt
done
timeout -k 10 240 python3 tools/stream_probe.py 10 > $O/stream_probe.txt 2>&1
