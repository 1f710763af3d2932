# round-4: wide GEMM tiles in XCD-contiguous runs with a panel's row tiles adjacent (default) vs
# the 2-D grid (OSW_WIDE_REMAP=0): GEMM kernel tests, beam-5 bench A/B, one-lane beam pass kernel times
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_ae; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_turbo.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 2 --warmup 1 --beam5-steps 6 --latency-repeats 0 --beam5-latency-repeats 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for v in 1 0; do
    OSW_WIDE_REMAP=$v timeout -k 10 400 python -u bench.py $A > $O/r${v}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/r${v}_$r.json'));print('remap$v run$r beam5',d['beam5']['value'],d['beam5'].get('ms_per_step'))"
  done
done
