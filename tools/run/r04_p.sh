# round-4: where the 8-phase GEMM's fp16 epilogue time goes (debug variants 9/12/13/8/10)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_p; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 300 python3 -u tools/probe/gemm_epi_probe.py 9,12,13,8,14,10,15 2 > $O/epi.jsonl 2> $O/epi.err
cat $O/epi.jsonl
