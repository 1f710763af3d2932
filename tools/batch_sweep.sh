# throughput at other batch / lane counts (exploration; the headline stays at 64 clips per step)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sweep}; mkdir -p $O
for cfg in "64 3" "128 2" "96 3" "192 2"; do
  set -- $cfg
  timeout -k 10 240 python -u bench.py --batch $1 --lanes $2 --steps 6 --beam5 0 --latency-repeats 1 --no-cpu-baseline > $O/b$1_l$2.json 2> $O/b$1_l$2.err
done
