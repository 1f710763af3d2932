# round-4: 8-phase GEMM epilogue with transposed accumulators (8-B / 16-B image writes)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_s; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 400 python3 -u tools/probe/gemm_epi_probe.py 9,8,16,10,17,19,18 2 > $O/epi.jsonl 2> $O/epi.err
cat $O/epi.jsonl
