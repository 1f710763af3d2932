# GPU tests (all, or -k EXPR) then bench + profile.  usage: gpu_check.sh OUT [pytest -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-check}; mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
bash tools/gpu_bench.sh ${1:-check}
