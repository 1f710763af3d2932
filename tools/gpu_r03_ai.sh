# config 5: small encoders skipping the encoder baton (OSW_BATON_MIN_WINDOWS=n) vs always
# serialised: streaming GPU test with the switch, then the 32-session simulation and the
# 4-caller probe, interleaved
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ai; mkdir -p $O
OSW_BATON_MIN_WINDOWS=9 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stream or sibling or concurrent" > $O/gpu_tests_bmin.log 2>&1
tail -1 $O/gpu_tests_bmin.log
A="--steps 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline"
for r in 1; do
  for E in "X=0" "OSW_BATON_MIN_WINDOWS=9" "OSW_BATON_MIN_WINDOWS=3"; do
    env $E timeout -k 10 300 python -u bench.py $A > $O/b.json 2> $O/b.err
    python3 -c "import json;d=json.load(open('$O/b.json'));s=d['streaming'];print('$E','run $r',d['value'],s['transcriptions_per_s'],s['call_latency_p50_ms'],s['final_transcript_lag_p50_s'])"
  done
done
for E in "X=0" "OSW_BATON_MIN_WINDOWS=9"; do
  echo "== $E"; env $E timeout -k 10 300 python -u tools/stream_probe.py 10 > $O/probe.txt 2>&1; cat $O/probe.txt
done
