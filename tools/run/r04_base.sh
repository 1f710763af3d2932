# round-4 first GPU call: GPU suite, default bench, cross-attention half-key A/B,
# rocprofv3 concurrent-caller probe (the round-3 SIGSEGV)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_base; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log
# 1 = some tests failed (keep going); anything else but 0 = stop here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stop"; exit $rc; fi
set -e
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
head -c 1500 $O/bench.json; echo
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for L in open-speech_amd/lib/libosw_hip.so open-speech_amd/lib/exp/libosw_xhalf.so; do
  OSW_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/ab.json 2> $O/ab.err
  python3 -c "import json;d=json.load(open('$O/ab.json'));print('$L',d['value'],d['ms_per_step'])"
done
export TMPDIR=/tmp
set +e
PYTHONFAULTHANDLER=1 OSW_TRACE_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/stream_probe.py 3 > $O/stream_probe_prof.txt 2>&1
echo "profiled concurrent probe rc $?"; tail -30 $O/stream_probe_prof.txt
