# round-4: REST-style concurrent load, batcher gap 1 ms (default) vs 1000 ms (= wait the full
# STT_HIP_BATCH_WAIT_MS window), two runs each interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_m; mkdir -p $O
set -e
for r in 1 2; do
  STT_HIP_BATCH_GAP_MS=1 timeout -k 10 300 python3 -u tools/rest_probe.py 16 6 40 >> $O/rest.txt 2> $O/rest1.err
  STT_HIP_BATCH_GAP_MS=1000 timeout -k 10 300 python3 -u tools/rest_probe.py 16 6 40 >> $O/rest.txt 2> $O/rest2.err
done
cat $O/rest.txt
