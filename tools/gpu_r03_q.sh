# ring128 + 64-query attention first look: GPU suite, small-M GEMM variants, small-batch encoder profile, streaming probe
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 tools/small_gemm_bench.py 1,2,4,8 > $O/small_gemm.jsonl 2>&1
bash tools/gpu_small_batch.sh r03_q/sb
