# round-4: transposed accumulators for the fp16 epilogues only (fp32 / head-major kernels back
# to <= 216 VGPRs): parity subset, headline x2 with beam 5
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_u; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  timeout -k 10 400 python -u bench.py $A > $O/h$r.json 2> $O/h.err
  python3 -c "import json;d=json.load(open('$O/h$r.json'));print('h$r',d['value'],d['ms_per_step'],d['beam5']['value'],d['stages_ms_roofline_pass']['encoder_gemm'])"
done
