# GPU tests (optionally -k EXPR), then the bench twice: as built, and with one
# environment switch (A/B in one call; streaming leg skipped).  usage: gpu_ab_bench.sh OUT VAR=VALUE [pytest -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abb}; mkdir -p $O
if [ -n "$3" ]; then K=(-k "$3"); else K=(); fi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --stream-sessions 0 --realistic-steps 0 --latency-repeats 10 --beam5-latency-repeats 10 > $O/bench_a.json 2> $O/bench_a.err
env $2 timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --stream-sessions 0 --realistic-steps 0 --latency-repeats 10 --beam5-latency-repeats 10 > $O/bench_b.json 2> $O/bench_b.err
