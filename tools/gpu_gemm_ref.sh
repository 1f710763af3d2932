# torch.matmul vs our GEMM on the encoder shapes.  usage: gpu_gemm_ref.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-gref}; mkdir -p $O
timeout -k 10 200 python -u tools/torch_gemm_ref.py > $O/torch.txt 2>&1
timeout -k 10 200 python -u tools/gemm_bench.py enc > $O/ours.txt 2>&1
