# round-4 checkpoint: the whole GPU suite, the default bench, a one-lane kernel-trace profile,
# the PMC traffic passes (profiles/r04_*), and the concurrent-caller probe under the profiler
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
set -e
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_b1'],d['beam5']['value'],d['realistic_lengths']['value'],d['streaming']['transcriptions_per_s'])"
B="--steps 3 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $B > $O/prof.json 2> $O/prof.err
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 25 > $O/kernel_summary.txt; head -12 $O/kernel_summary.txt
rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 700 bash tools/pmc_run.sh r04_k/pmc
set +e
STREAM_PROBE_MAPS=$O/maps.txt PYTHONFAULTHANDLER=1 OSW_TRACE_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sprof -o run -- python3 tools/stream_probe.py 3 > $O/stream_probe_prof.txt 2>&1
echo "profiled concurrent probe rc $?"
rm -f $O/sprof/run_kernel_trace.csv
exit 0
