# SQ counters per kernel (VALU / memory-wait / LDS picture) over one 1-lane greedy step and
# one beam-5 step: one rocprofv3 --pmc pass per counter group, summarised on the box.
# usage: pmc_sq_run.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmcsq}; mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --lanes 1 --beam5 1 --beam5-steps 0 --latency-repeats 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 bench.py $ARGS > $O/a.log 2>&1
python3 tools/pmc_generic.py $O/a/run_counter_collection.csv > $O/sq_summary.txt
rm -f $O/a/run_counter_collection.csv
