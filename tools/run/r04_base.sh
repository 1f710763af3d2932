# round-4 baseline on a fresh box: GPU suite + default bench
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_base; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -2 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json | head -c 3000
# experiment: headline with the cross-attention reading half the keys (timing only)
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for L in open-speech_amd/lib/libosw_hip.so open-speech_amd/lib/exp/libosw_xhalf.so; do
  OSW_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/ab.json 2> $O/ab.err
  python3 -c "import json;d=json.load(open('$O/ab.json'));print('$L',d['value'],d['ms_per_step'])"
done
