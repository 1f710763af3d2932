# round-4: pair cross-attention without prefetch capped at 80 VGPRs (fits beside an encoder
# workgroup): greedy tests with it on, the probe alone, 3-lane headline A/B interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_x; mkdir -p $O
export TMPDIR=/tmp
set -e
OSW_XATTN_PAIR=1 OSW_XATTN_PAIR_PF=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 ./tools/probe/xattn_probe > $O/probe.txt 2>&1
grep -E "product|pair|stream" $O/probe.txt
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/chunk_$r.json 2> $O/h.err
  OSW_XATTN_PAIR=1 OSW_XATTN_PAIR_PF=0 timeout -k 10 300 python -u bench.py $A > $O/pair0_$r.json 2> $O/h.err
  for v in chunk pair0; do
    python3 -c "import json;d=json.load(open('$O/${v}_$r.json'));print('$v run$r',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['frac'])"
  done
done
