# round-4: greedy cross-attention pair kernel: parity tests, then the headline A/B (chunk kernel,
# pair kernel without / with prefetch), two runs each interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_j; mkdir -p $O
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_turbo.py tests/test_gpu_refill.py > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  OSW_XATTN_PAIR=0 timeout -k 10 300 python -u bench.py $A > $O/chunk$r.json 2> $O/chunk.err
  OSW_XATTN_PAIR_PF=0 timeout -k 10 300 python -u bench.py $A > $O/pair$r.json 2> $O/pair.err
  timeout -k 10 300 python -u bench.py $A > $O/pairpf$r.json 2> $O/pairpf.err
  for f in chunk$r pair$r pairpf$r; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'])"; done
done
