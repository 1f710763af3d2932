# GPU tests under an environment switch + isolated-pass A/B of that switch.  usage: gpu_ab2.sh OUT "pytest -k expr" VAR=VALUE
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab2}; mkdir -p $O
env $3 timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$2" > $O/gpu_tests.log 2>&1
timeout -k 10 240 python -u bench.py --steps 6 --beam5-steps 0 --beam5 0 --no-cpu-baseline > $O/bench_a.json 2> $O/bench_a.err
env $3 timeout -k 10 240 python -u bench.py --steps 6 --beam5-steps 0 --beam5 0 --no-cpu-baseline > $O/bench_b.json 2> $O/bench_b.err
