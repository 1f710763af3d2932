# round-4: phased lanes (decode chunks wait for the last enqueued encoder; encoders on the whole
# grid), with and without the E-form cross-attention, against the default, interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ab; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/def_$r.json 2> $O/h.err
  OSW_PHASED=1 timeout -k 10 300 python -u bench.py $A > $O/ph_$r.json 2> $O/h.err
  OSW_PHASED=1 OSW_EFORM=1 timeout -k 10 300 python -u bench.py $A > $O/phe_$r.json 2> $O/h.err
  for v in def ph phe; do
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v run$r',d['value'],d['ms_per_step'])"
  done
done
