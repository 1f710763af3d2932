# round-4: lanes per GPU (2 / 3 / 4) on the headline, interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ah; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for l in 3 4 2; do
    timeout -k 10 400 python -u bench.py $A --lanes $l > $O/l${l}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/l${l}_$r.json'));print('lanes $l run$r',d['value'],d['ms_per_step'])"
  done
done
