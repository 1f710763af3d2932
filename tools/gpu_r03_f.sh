set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03_f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "robustness or parity or turbo or kernels" > gpurun_out/r03_f/gpu_tests.log 2>&1
tail -1 gpurun_out/r03_f/gpu_tests.log
bash tools/gpu_ab_prof.sh r03_f_prof "OSW_SKINNY_NOPRE=1 OSW_SKINNY_NOPAIR=1 OSW_GEMM_NEXT0=0 OSW_NO_FUSE_SELECT=1 OSW_ATTN_LAZY=0"
BENCH_ARGS="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_f_ab "OSW_X=0" "OSW_GEMM_NEXT0=0" "OSW_SKINNY_NOPAIR=1" "OSW_ATTN_LAZY=0"
BENCH_ARGS="--steps 1 --warmup 1 --latency-repeats 30 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_f_lat "OSW_X=0" "OSW_NO_FUSE_SELECT=1"
