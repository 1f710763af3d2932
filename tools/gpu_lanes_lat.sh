# lanes sweep (20 steps) and a batch-1 latency A/B over OSW_LOGITS_SPLIT.  usage: gpu_lanes_lat.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
Q="--latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
for L in 4 2; do
  timeout -k 10 300 python -u bench.py --lanes $L --steps 20 $Q > $O/l$L.json 2> $O/l$L.err
  python3 -c "import json;print('lanes', $L, json.load(open('$O/l$L.json'))['value'])"
done
for r in 1 2; do for S in 0 1; do
  OSW_LOGITS_SPLIT=$S timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --latency-repeats 50 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline > $O/lat$S_$r.json 2> $O/lat$S.err
  python3 -c "import json;d=json.load(open('$O/lat$S_$r.json'));print('logits_split', $S, d['latency_b1']['greedy'])"
done; done
