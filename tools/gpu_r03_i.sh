set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03_i
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "encoder or tile or turbo_encoder or tiny_encoder or batch_equals" > gpurun_out/r03_i/gpu_tests.log 2>&1
tail -1 gpurun_out/r03_i/gpu_tests.log
BENCH_ARGS="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_i_ab "OSW_X=0" "OSW_ATTN_GRID=1000000" "OSW_ATTN_GRID=256" "OSW_ATTN_GRID=512"
