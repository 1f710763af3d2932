# confirmation of the committed tree: whole GPU suite, default bench line
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));s=d['streaming'];print(d['value'],d['roofline']['frac'],(d.get('beam5') or {}).get('value'),d['latency_b1'],s['transcriptions_per_s'],s['final_transcript_lag_p50_s'])"
