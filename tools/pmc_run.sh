# HBM traffic per kernel: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short
# 1-lane bench, summarised on the box by pmc_summary.py.  usage: pmc_run.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmc}; mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --lanes 1 --beam5 0 --beam5-steps 0 --latency-repeats 0 --beam5-latency-repeats 0 --stream-sessions 0 --rest-callers 0 --realistic-steps 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 bench.py $ARGS > $O/f.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 bench.py $ARGS > $O/w.log 2>&1
python3 tools/pmc_summary.py $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv $O/pmc.json
rm -f $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv
