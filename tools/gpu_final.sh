# Round-end evidence for the tree as committed: the whole GPU suite, the default bench line,
# a rocprofv3 kernel trace (+ --stats) of a short bench, and the two PMC traffic passes.
# usage: gpu_final.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['kernel'],d['roofline']['frac'],(d.get('beam5') or {}).get('value'),d.get('p50_latency_ms_b1'))"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline --latency-repeats 5 --beam5-latency-repeats 3 --stream-sessions 0 --realistic-steps 0 > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/trace_summary.py $O/prof/run_kernel_trace.csv $O/s 18 1
gzip -f $O/prof/run_kernel_trace.csv
bash tools/pmc_run.sh ${1:-final}_pmc
