# beam rows' split-K projections on the 64 x 256 tile too (OSW_WIDE256_ALL=1) vs 64 x 128
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ah; mkdir -p $O
OSW_WIDE256_ALL=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "beam or stream or batch" > $O/gpu_tests_all256.log 2>&1
tail -1 $O/gpu_tests_all256.log
bash tools/gpu_ab_prof.sh r03_ah_prof OSW_WIDE256_ALL=1
grep -h "gemm_wide" gpurun_out/r03_ah_prof/a_beam5* gpurun_out/r03_ah_prof/b_beam5* || true
BENCH_ARGS="--steps 6 --latency-repeats 0 --beam5-latency-repeats 10 --beam5 1 --beam5-steps 3 --stream-sessions 0 --realistic-steps 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_ah_ab "X=0" "OSW_WIDE256_ALL=1"
