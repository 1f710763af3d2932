# GEMM K sweep (per-tile overhead) for the 8-phase kernel: fp32 out, fp16 out, GELU fp16
# out, no epilogue.  usage: gpu_ksweep.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ks}; mkdir -p $O
for v in 4 8 10 9; do
  KS=1280,2560 timeout -k 10 200 python -u tools/gemm_ksweep.py $v > $O/ksweep_v$v.txt 2>&1
done
