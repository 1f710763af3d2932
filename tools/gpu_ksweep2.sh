# 8-phase GEMM on the guide's square shapes (4096^3, 8192^3): fp32 out vs no epilogue.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ks}; mkdir -p $O
for v in 4 9; do
  KS=4096 timeout -k 10 200 python -u tools/gemm_ksweep.py $v 4096 4096 > $O/sq4k_v$v.txt 2>&1
  KS=8192 timeout -k 10 200 python -u tools/gemm_ksweep.py $v 8192 8192 > $O/sq8k_v$v.txt 2>&1
done
