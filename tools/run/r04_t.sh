# round-4: transposed 8-phase accumulators + pinned GELU rounding: GPU suite, epilogue forms, headline
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_t; mkdir -p $O
export TMPDIR=/tmp
set -e
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 -u tools/probe/gemm_epi_probe.py 9,8,12,10,13,15,14 2 > $O/epi.jsonl 2> $O/epi.err
cat $O/epi.jsonl
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/h$r.json 2> $O/h.err
  python3 -c "import json;d=json.load(open('$O/h$r.json'));print('h$r',d['value'],d['ms_per_step'],d['stages_ms_roofline_pass'])"
done
