set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_h_ab "OSW_X=0" "OSW_GEMM_GRID=128" "OSW_GEMM_GRID=176" "OSW_ENC_BATON=0"
BENCH_ARGS="--steps 10 --lanes 4 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_h_l4 "OSW_X=0"
BENCH_ARGS="--steps 1 --warmup 1 --latency-repeats 30 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_h_lat "OSW_X=0" "OSW_NO_FUSE_SELECT=1"
