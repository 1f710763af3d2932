# beam cross-attention K through LDS (whole-line loads) vs direct fragment loads
set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--steps 2 --latency-repeats 0 --beam5 1 --beam5-steps 4 --beam5-latency-repeats 10 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" \
  PRE_TESTS="beam or sibling or batch" bash tools/gpu_env_ab.sh r03_aa "OSW_KLDS=1" "OSW_XATTN_KDIRECT=1"
grep -h "dec_xattn_mfma\|beam5" gpurun_out/r03_aa/bench_1_1.json | head -2 > /dev/null || true
