# bench A/B over environment settings.  usage: gpu_env_ab.sh OUT "ENV1" "ENV2" ...  (each ENV like "A=1 B=0")
# BENCH_ARGS overrides the bench arguments; PRE_TESTS (pytest -k expr, or all) runs those GPU tests first.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --stream-sessions 0 --no-cpu-baseline"}
if [ -n "$PRE_TESTS" ]; then
  if [ "$PRE_TESTS" = all ]; then K=(); else K=(-k "$PRE_TESTS"); fi
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
  tail -2 $O/gpu_tests.log
fi
for r in 1 2; do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 300 python -u bench.py $ARGS > $O/bench_${i}_$r.json 2> $O/bench_${i}_$r.err
    python3 -c "import json;d=json.load(open('$O/bench_${i}_$r.json'));b=d.get('beam5') or {};rl=d.get('realistic_lengths') or {};lat=d.get('latency_b1') or {};print('$E','run',$r,d['value'],b.get('value'),rl.get('value'),(lat.get('greedy') or {}).get('p50_ms'),(lat.get('beam5') or {}).get('p50_ms'))"
  done
done
