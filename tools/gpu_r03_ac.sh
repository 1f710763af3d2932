# headline vs timed-step count (pipeline fill over the 3 lanes) and lane count
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ac; mkdir -p $O
A="--latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --stream-sessions 0 --realistic-steps 0 --no-cpu-baseline"
for r in 1 2; do
for cfg in "--steps 6" "--steps 12" "--steps 24" "--steps 12 --lanes 4" "--steps 12 --lanes 2"; do
  timeout -k 10 300 python -u bench.py $A $cfg > $O/b.json 2> $O/b.err
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$cfg', 'run $r', d['value'], d['ms_per_step'])"
done
done
