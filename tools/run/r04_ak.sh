# round-4: poll-ahead decode loop (the next graph chunk is enqueued before the host reads the
# done count) vs OSW_POLL_AHEAD=0: parity/beam/backend tests, p50 and headline A/B interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ak; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py tests/test_gpu_refill.py tests/test_gpu_backend.py tests/test_gpu_longform.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 12 --latency-repeats 30 --beam5-latency-repeats 10 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for v in 1 0; do
    OSW_POLL_AHEAD=$v timeout -k 10 400 python -u bench.py $A > $O/p${v}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/p${v}_$r.json'));print('poll_ahead $v run$r',d['value'],d['p50_latency_ms_b1'],d.get('p50_latency_ms_b1_beam5'))"
  done
done
