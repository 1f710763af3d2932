# round-4 call: E-form headline A/B + one-lane kernel times
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_g; mkdir -p $O
export TMPDIR=/tmp
set -e
OSW_EFORM=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_gpu_turbo.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
OSW_EFORM=1 timeout -k 10 300 python -u bench.py $A > $O/eform$r.json 2> $O/eform.err
OSW_EFORM=0 timeout -k 10 300 python -u bench.py $A > $O/noeform$r.json 2> $O/noeform.err
for f in eform$r noeform$r; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['ms_per_step'],d['tokens_per_clip'])"; done
done
B="--steps 3 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
OSW_EFORM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ef -o run -- python3 bench.py $B > $O/ef.json 2> $O/ef.err
python3 tools/kstats.py $O/ef/run_kernel_stats.csv 16
rm -f $O/*/run_kernel_trace.csv
