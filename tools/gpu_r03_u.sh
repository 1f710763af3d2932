# A/B: direct skinny (logits) kernels at 4 waves/SIMD (one round of 811 workgroups) vs default
set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--steps 1 --warmup 0 --latency-repeats 30 --beam5 0 --beam5-steps 0 --beam5-latency-repeats 10 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" \
  PRE_TESTS="turbo or batch1 or fused" bash tools/gpu_lib_ab.sh r03_u open-speech_amd/lib/libosw_hip.so open-speech_amd/lib/ab/libosw_wpe4.so
