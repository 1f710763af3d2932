# batch-1 logits: second weight chunk issued before the prologue (4 waves/EU) vs after
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "turbo or batch or fused or robust or nan" > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
for i in 1 2; do
timeout -k 10 120 python3 tools/latency_probe.py 40 1 > $O/lat_early_$i.txt 2>&1
OSW_PRO_WB_LATE=1 timeout -k 10 120 python3 tools/latency_probe.py 40 1 > $O/lat_late_$i.txt 2>&1
done
grep -H p50 $O/lat_*.txt
