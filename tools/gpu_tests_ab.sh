# GPU tests (-k EXPR, or all) then a bench A/B over environment settings in the same call.
# usage: gpu_tests_ab.sh OUT "pytest -k expr|all" "ENV1" "ENV2" ...
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; K=$2; shift 2; mkdir -p $O
if [ "$K" = all ]; then KA=(); else KA=(-k "$K"); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
PRE_TESTS= bash tools/gpu_env_ab.sh $(basename $O)_ab "$@"
