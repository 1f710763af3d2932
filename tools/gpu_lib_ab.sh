# bench A/B over library builds (OSW_LIB).  usage: gpu_lib_ab.sh OUT LIB1 LIB2 ...  (paths relative to the repo)
# BENCH_ARGS overrides the bench arguments; PRE_TESTS (pytest -k expr) runs those GPU tests first (default library).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift; mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 3 --latency-repeats 0 --beam5 1 --beam5-steps 4 --beam5-latency-repeats 10 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline"}
if [ -n "$PRE_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PRE_TESTS" > $O/gpu_tests.log 2>&1
  tail -1 $O/gpu_tests.log
fi
for r in 1 2; do
  i=0
  for L in "$@"; do
    i=$((i+1))
    OSW_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 400 python -u bench.py $ARGS > $O/bench_${i}_$r.json 2> $O/bench_${i}_$r.err
    python3 -c "import json;d=json.load(open('$O/bench_${i}_$r.json'));b=d.get('beam5') or {};lat=d.get('latency_b1') or {};print('$L','run',$r,d['value'],b.get('value'),d.get('beam5_audio_sec_per_sec_1lane'),(lat.get('greedy') or {}).get('p50_ms'),(lat.get('beam5') or {}).get('p50_ms'))"
  done
done
