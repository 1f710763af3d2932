# Headline throughput at 2, 3 and 4 lanes per GPU (greedy leg only).  usage: gpu_lanes.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-lanes}; mkdir -p $O
for n in 3 2 4; do
  timeout -k 10 300 python -u bench.py --steps 6 --lanes $n --no-cpu-baseline --beam5 0 --beam5-steps 0 --latency-repeats 0 --beam5-latency-repeats 0 --stream-sessions 0 --realistic-steps 0 > $O/bench_l$n.json 2> $O/bench_l$n.err
done
