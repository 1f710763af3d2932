# round-4: greedy cross-attention in 16 key chunks per (window, head) (OSW_XATTN_CHUNKS=16) vs 8:
# greedy tests with 16, then headline + batch-1 p50 + roofline pass, interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_af; mkdir -p $O
export TMPDIR=/tmp
set -e
OSW_XATTN_CHUNKS=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py tests/test_gpu_refill.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 12 --latency-repeats 20 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for c in 8 16; do
    OSW_XATTN_CHUNKS=$c timeout -k 10 400 python -u bench.py $A > $O/c${c}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/c${c}_$r.json'));print('chunks $c run$r',d['value'],d['ms_per_step'],d['p50_latency_ms_b1'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
  done
done
