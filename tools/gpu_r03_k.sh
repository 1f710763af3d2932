set -e
cd "$GRAFT_REPO_ROOT"
PRE_TESTS="beam" bash tools/gpu_lib_ab.sh r03_k open-speech_amd/lib/ab/libosw_base.so open-speech_amd/lib/libosw_hip.so open-speech_amd/lib/ab/libosw_x6.so
BENCH_ARGS="--steps 8 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_k_stag "OSW_GEMM_STAGGER=0" "OSW_GEMM_STAGGER=3" "OSW_GEMM_STAGGER=6"
for f in gpurun_out/r03_k_stag/bench_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',d['rooflines']['encoder_gemm'])"; done
