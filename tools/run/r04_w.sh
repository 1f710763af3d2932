# round-4 final checkpoint: the whole GPU suite, the default bench, a one-lane kernel-trace
# profile and the PMC traffic passes of the committed tree (profiles/r04_w_*)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
set -e
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['p50_latency_ms_b1'],d['beam5']['value'],d['realistic_lengths']['value'],d['streaming']['transcriptions_per_s'],d['roofline'])"
B="--steps 3 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py $B > $O/prof.json 2> $O/prof.err
python3 tools/kstats.py $O/prof/run_kernel_stats.csv 25 > $O/kernel_summary.txt; head -8 $O/kernel_summary.txt
rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 700 bash tools/pmc_run.sh r04_w/pmc
echo done
