# fragment-major decoder weights: GPU suite, then bench A/B against the row-major stream
set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--steps 6 --latency-repeats 30 --beam5 1 --beam5-steps 4 --beam5-latency-repeats 10 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" \
  PRE_TESTS=all bash tools/gpu_env_ab.sh r03_x2 "OSW_WFRAG=1" "OSW_NO_WFRAG=1"
