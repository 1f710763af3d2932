set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--steps 10 --latency-repeats 0 --beam5 0 --beam5-steps 0 --beam5-latency-repeats 0 --realistic-steps 6 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_o "OSW_X=0" "OSW_GEMM_GRID=224" "OSW_GEMM_GRID=256"
