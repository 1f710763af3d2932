# round-4: GEMM kernel tests incl. the transposed-epilogue bit identity
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ac; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
