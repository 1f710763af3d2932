# round-4: encoder attention with a 4-slot K/V ring: parity tests, headline, one-lane kernel times
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_n; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_turbo.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -50 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/ring$r.json 2> $O/ring.err
  python3 -c "import json;d=json.load(open('$O/ring$r.json'));print('ring$r',d['value'],d['ms_per_step'],d['stages_ms_roofline_pass']['encoder_attention'])"
done
B="--steps 3 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $B > $O/prof.json 2> $O/prof.err
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 12
rm -f $O/prof/run_kernel_trace.csv
