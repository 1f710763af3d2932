# beam candidate lists by threshold + rank (default) vs K2 block-wide pops (OSW_BEAM_POPS=1):
# beam tests, kernel traces of the isolated passes, beam-5 throughput / batch-1 latency A/B
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_af; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "beam or stream" > $O/gpu_tests_beam.log 2>&1
tail -1 $O/gpu_tests_beam.log
bash tools/gpu_ab_prof.sh r03_af_prof OSW_BEAM_POPS=1
grep -h "select_kernel\|beam_update" gpurun_out/r03_af_prof/a* gpurun_out/r03_af_prof/b* || true
BENCH_ARGS="--steps 6 --latency-repeats 0 --beam5-latency-repeats 20 --beam5 1 --beam5-steps 3 --stream-sessions 0 --realistic-steps 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_af_ab "X=0" "OSW_BEAM_POPS=1"
