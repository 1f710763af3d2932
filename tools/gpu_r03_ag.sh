# logits GEMM on a 64 x 256 tile (8 waves, default) vs 64 x 128 (OSW_WIDE_N128=1): whole GPU
# suite, kernel traces of the isolated passes, greedy / beam-5 / batch-1 A/B
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
bash tools/gpu_ab_prof.sh r03_ag_prof OSW_WIDE_N128=1
grep -h "gemm_wide" gpurun_out/r03_ag_prof/a* gpurun_out/r03_ag_prof/b* || true
BENCH_ARGS="--steps 12 --latency-repeats 30 --beam5-latency-repeats 10 --beam5 1 --beam5-steps 3 --stream-sessions 0 --realistic-steps 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_ag_ab "X=0" "OSW_WIDE_N128=1"
