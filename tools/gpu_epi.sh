# GEMM epilogue check: kernel tests, K sweep of the fp16 / GELU / no-epilogue variants, bench.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-epi}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "kernels or parity or turbo" > $O/gpu_tests.log 2>&1
for v in 10 8 9; do
  KS=1280,2560 timeout -k 10 200 python -u tools/gemm_ksweep.py $v > $O/ksweep_v$v.txt 2>&1
done
timeout -k 10 300 python -u bench.py --steps 6 --no-cpu-baseline --beam5 0 --beam5-steps 0 --latency-repeats 0 --beam5-latency-repeats 0 --stream-sessions 0 --realistic-steps 0 > $O/bench.json 2> $O/bench.err
