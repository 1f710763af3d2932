# round-4: 8-phase GEMM stagger sweep; then the concurrent-caller probe under rocprofv3 with the maps dump
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_h; mkdir -p $O
export TMPDIR=/tmp
set -e
for s in 0 20000 40000 60000 0; do
  OSW_GEMM_STAGGER=$s timeout -k 10 200 python3 -u tools/probe/gemm_stagger.py >> $O/stagger.jsonl 2> $O/stagger.err
done
cat $O/stagger.jsonl
set +e
STREAM_PROBE_MAPS=$O/maps.txt PYTHONFAULTHANDLER=1 OSW_TRACE_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/stream_probe.py 3 > $O/stream_probe_prof.txt 2>&1
echo "profiled concurrent probe rc $?"; grep -n "SIGSEGV\|calls/s\|sequential" $O/stream_probe_prof.txt | head
rm -f $O/prof/run_kernel_trace.csv
exit 0
