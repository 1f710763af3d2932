# round-4: A/B in one call, fp16 epilogues with transposed accumulators (default) vs plain (OSW_GEMM_TR=0)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_v; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for tr in 1 0; do
    OSW_GEMM_TR=$tr timeout -k 10 300 python -u bench.py $A > $O/tr${tr}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/tr${tr}_$r.json'));print('tr$tr run$r',d['value'],d['ms_per_step'],d['stages_ms_roofline_pass']['encoder_gemm'])"
  done
done
