# fused batch-1 selection with the select state preloaded: GPU suite + batch-1 latency
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 120 python3 tools/latency_probe.py 30 1 > $O/lat1_$i.txt 2>&1
OSW_NO_FUSE_SELECT=1 timeout -k 10 120 python3 tools/latency_probe.py 30 1 > $O/lat1_nofuse_$i.txt 2>&1
done
grep -h "p50" $O/lat1_*.txt
