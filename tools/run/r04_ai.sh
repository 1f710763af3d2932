# round-4: kernel tests + parity after removing the unused fp32 transposed epilogue branches
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ai; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_turbo.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
