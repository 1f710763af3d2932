# round-4 call 2: timing experiments (what the 3-lane headline is sensitive to) and the
# rocprofv3 graph-launch crash (minimal reproducer; the probe without graphs)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_b; mkdir -p $O
set -e
A="--steps 10 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for L in open-speech_amd/lib/libosw_hip.so open-speech_amd/lib/exp/libosw_noln.so open-speech_amd/lib/exp/libosw_enchalf.so open-speech_amd/lib/exp/libosw_xhalf.so open-speech_amd/lib/libosw_hip.so; do
  OSW_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/ab.json 2> $O/ab.err
  python3 -c "import json;d=json.load(open('$O/ab.json'));print('$L',d['value'],d['ms_per_step'],d['tokens_per_clip'])"
done
export TMPDIR=/tmp
set +e
timeout -k 10 120 ./tools/graph_prof_repro 3 300 1 > $O/repro_plain.txt 2>&1; echo "repro without profiler rc $?"; tail -2 $O/repro_plain.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_repro -o run -- ./tools/graph_prof_repro 3 300 1 > $O/repro_prof.txt 2>&1; echo "repro under rocprofv3 kernel-trace rc $?"; tail -25 $O/repro_prof.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_repro0 -o run -- ./tools/graph_prof_repro 3 300 0 > $O/repro_prof0.txt 2>&1; echo "repro (no concurrent capture) under rocprofv3 rc $?"; tail -5 $O/repro_prof0.txt
OSW_NO_GRAPH=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nograph -o run -- python3 tools/stream_probe.py 3 > $O/stream_probe_nograph_prof.txt 2>&1; echo "probe OSW_NO_GRAPH=1 under rocprofv3 rc $?"; tail -5 $O/stream_probe_nograph_prof.txt
exit 0
