# GPU test suite (all, or -k EXPR).  usage: gpu_tests.sh OUT [pytest -k expr]
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-tests}; mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1
