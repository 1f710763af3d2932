# self-attention V prefetch (OSW_SELF_VPRE=1): parity tests with the switch, kernel traces
# of the isolated passes, headline / batch-1 latency / beam-5 A/B
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ae; mkdir -p $O
OSW_SELF_VPRE=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "turbo or beam or parity or batch" > $O/gpu_tests_vpre.log 2>&1
tail -1 $O/gpu_tests_vpre.log
bash tools/gpu_ab_prof.sh r03_ae_prof OSW_SELF_VPRE=1
grep -h self_attn gpurun_out/r03_ae_prof/a* gpurun_out/r03_ae_prof/b* || true
BENCH_ARGS="--steps 12 --latency-repeats 30 --beam5-latency-repeats 10 --beam5 1 --stream-sessions 0 --realistic-steps 0 --no-cpu-baseline" bash tools/gpu_env_ab.sh r03_ae_ab "X=0" "OSW_SELF_VPRE=1"
