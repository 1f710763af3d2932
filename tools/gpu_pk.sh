# Packed-FP32 re-enable check: the library built with v_pk_*_f32 (make NOPK= BUILD=build_pk
# OUT=../lib/libosw_hip_pk.so) under the interference probe (a second context loops each
# stage while the first decodes; results must stay bit-identical), the concurrent-lane GPU
# tests, and the bench against the default library.  usage: gpu_pk.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pk}; mkdir -p $O
PK=$PWD/open-speech_amd/lib/libosw_hip_pk.so
OSW_LIB=$PK timeout -k 10 400 python -u tools/interference_probe.py > $O/interference_pk.txt 2>&1
OSW_LIB=$PK timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "sibling or concurrent or parity" > $O/gpu_tests_pk.log 2>&1
timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --stream-sessions 0 --realistic-steps 0 --latency-repeats 10 --beam5-latency-repeats 10 > $O/bench_a.json 2> $O/bench_a.err
OSW_LIB=$PK timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --stream-sessions 0 --realistic-steps 0 --latency-repeats 10 --beam5-latency-repeats 10 > $O/bench_pk.json 2> $O/bench_pk.err
