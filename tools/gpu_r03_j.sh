set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "encoder or tile or turbo_encoder or tiny_encoder or batch_equals or lanes or sibling" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline > $O/bench_$r.json 2> $O/bench_$r.err
  python3 -c "import json;d=json.load(open('$O/bench_$r.json'));r=d['roofline'];print('run',$r,d['value'],r['achieved'],r['frac'],r['avg_launch_ms'])"
done
