# self-attention V prefetch up to 20 rows (config 5's 4 windows x 5 beams) vs up to 8
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ak; mkdir -p $O
OSW_SELF_VPRE_ROWS=20 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stream or beam" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
A="--steps 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline"
for r in 1 2; do
  for E in "X=0" "OSW_SELF_VPRE_ROWS=20"; do
    env $E timeout -k 10 300 python -u bench.py $A > $O/b.json 2> $O/b.err
    python3 -c "import json;d=json.load(open('$O/b.json'));s=d['streaming'];print('$E','run $r',s['transcriptions_per_s'],s['call_latency_p50_ms'],s['final_transcript_lag_p50_s'])"
  done
done
