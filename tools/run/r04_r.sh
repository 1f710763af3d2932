# round-4: encoder attention forms (row sums by MFMA / VALU, -m as the C operand / VALU add,
# the previous product form), two score spreads
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_r; mkdir -p $O
set -e
timeout -k 10 120 ./tools/probe/attn_probe 64 4 > $O/attn_probe_s4.jsonl 2>&1
timeout -k 10 120 ./tools/probe/attn_probe 64 16 > $O/attn_probe_s16.jsonl 2>&1
cat $O/attn_probe_s4.jsonl $O/attn_probe_s16.jsonl
