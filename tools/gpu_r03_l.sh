set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03_l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_l/gpu_tests.log 2>&1
tail -1 gpurun_out/r03_l/gpu_tests.log
BENCH_ARGS="--steps 8 --latency-repeats 0 --beam5 1 --beam5-steps 4 --beam5-latency-repeats 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_lib_ab.sh r03_l_ab open-speech_amd/lib/ab/libosw_base.so open-speech_amd/lib/libosw_hip.so
