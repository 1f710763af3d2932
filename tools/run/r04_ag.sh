# round-4: 64-row greedy logits on the skinny kernel (fits beside an encoder workgroup;
# OSW_SKINNY_LOGITS=1) vs the 64 x 256 wide tile: greedy tests with it, headline A/B interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ag; mkdir -p $O
export TMPDIR=/tmp
set -e
OSW_SKINNY_LOGITS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for v in 0 1; do
    OSW_SKINNY_LOGITS=$v timeout -k 10 400 python -u bench.py $A > $O/s${v}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/s${v}_$r.json'));print('skinny_logits $v run$r',d['value'],d['ms_per_step'])"
  done
done
