# tile selection by count + staged square-tile epilogues: GPU suite, small-batch profile,
# streaming probe, then a short bench (headline, B=1 latency, config-5 streaming)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/gpu_small_batch.sh r03_r/sb
timeout -k 10 600 python3 bench.py --steps 6 --beam5 0 --beam5-steps 0 --realistic-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
