# round-4: row refill tests, the affected parity tests, then bench realistic lengths (refill vs not)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_i; mkdir -p $O
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_refill.py tests/test_gpu_parity.py tests/test_gpu_robustness.py > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 4 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --stream-sessions 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], json.dumps(d['realistic_lengths']))"
