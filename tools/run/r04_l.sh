# round-4: realistic lengths, row refill threshold sweep (9 steps, 3 lanes)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_l; mkdir -p $O
set -e
A="--steps 2 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --stream-sessions 0 --no-cpu-baseline --realistic-steps 9"
for m in 8 24 40 64; do
  timeout -k 10 400 python -u bench.py $A --refill-min $m > $O/r$m.json 2> $O/r$m.err
  python3 -c "import json;d=json.load(open('$O/r$m.json'))['realistic_lengths'];print('refill_min $m', d['value'], 'no refill', d['no_refill']['value'])"
done
