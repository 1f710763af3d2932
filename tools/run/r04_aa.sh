# round-4: 3-lane kernel-trace timeline (decoder kernel times beside an encoder vs alone)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_aa; mkdir -p $O
set -e
bash tools/gpu_trace.sh r04_aa
python3 tools/lane_timeline.py $O/prof/run_kernel_trace.csv.gz $O/timeline.txt
rm -f $O/prof/run_kernel_trace.csv.gz
head -80 $O/timeline.txt
