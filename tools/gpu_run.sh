#!/bin/bash
# One parameterised GPU runner (replaces the per-call tools/run/r04_*.sh scripts).
# usage: tools/gpu_run.sh TAG STEP [STEP ...]    (run through gpurun from the repo root)
# Every step has its own time limit; the first failing step ends the call.
#   tests       the whole -m gpu suite                      -> $O/gpu_tests.log
#   smoke       __graft_entry__.smoke()                     -> $O/smoke.log
#   t:FILES     selected gpu test files/ids (commas -> spaces) -> $O/t_N.log
#   bench       the default bench line                      -> $O/bench.json
#   prof        one-lane kernel trace of a 3-step bench     -> $O/kernel_summary.txt (+ stats csv)
#   pmc         FETCH_SIZE / WRITE_SIZE passes (tools/pmc_run.sh) -> $O/pmc/pmc.json
#   stream      config-5 simulation with host breakdown     -> $O/stream.json
#   streamprof  the same under a kernel trace, eager decode -> $O/stream_classes.txt
#   b1          batch-1 greedy step breakdown               -> $O/b1_breakdown.txt
#   b1beam      batch-1 beam-5 step breakdown               -> $O/b1beam_breakdown.txt
#   pmcb1beam   SQ counter passes over a batch-1 beam-5 call -> $O/pmc_b1beam_{1,2}.txt
#   pmcfetch:SCRIPT,ARGS  FETCH_SIZE per dispatch of $PMC_MATCH kernels over python3 SCRIPT ARGS -> $O/pmcfetch_N.txt
#   pmcenc      the same SQ passes over one 64-window greedy step -> $O/pmc_enc_{1,2}.txt
#   repro       tools/graph_prof_repro (mode 2) under a rocprofv3 kernel trace -> $O/repro.log
#   bench:ARGS  bench.py with extra args (commas -> spaces) -> $O/bench_N.json
#   py:SCRIPT,ARGS  python3 SCRIPT ARGS                     -> $O/py_N.txt
#   rprof:SCRIPT,ARGS  the same under a rocprofv3 kernel trace -> $O/rprof_N.txt, rprof_N.summary.txt
#   env:A=1,B=2 / unenv:A,B   set / clear environment variables for the following steps
# stream and streamprof write $O/stream[_prof]_N.json when run more than once (N = step index)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
QUICK="--latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline"
i=0
for s in "$@"; do
  i=$((i+1))
  echo "== step $i: $s ($(date +%T))"
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
      rc=$?; tail -5 $O/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
      rc=$?; tail -3 $O/smoke.log ;;
    t:*)
      A=${s#t:}; A=${A//,/ }
      timeout -k 10 900 python -u -m pytest $A -m gpu -v --timeout ${T_TIMEOUT:-300} --timeout-method thread -rf --durations=5 > $O/t_$i.log 2>&1
      rc=$?; tail -25 $O/t_$i.log ;;
    bench)
      timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
      [ $rc -eq 0 ] && python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d.get('p50_latency_ms_b1'),d.get('beam5',{}).get('value'),d.get('streaming',{}).get('transcriptions_per_s'),d['roofline']['frac'])" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --lanes 1 $QUICK > $O/prof.json 2> $O/prof.err
      rc=$?; [ $rc -eq 0 ] && python3 tools/kstats.py $O/prof/run_kernel_stats.csv 30 > $O/kernel_summary.txt && head -12 $O/kernel_summary.txt
      rm -f $O/prof/run_kernel_trace.csv ;;
    pmc)
      timeout -k 10 700 bash tools/pmc_run.sh $TAG/pmc; rc=$? ;;
    stream)
      timeout -k 10 300 python3 -u tools/stream_breakdown.py 32 6.0 $O/stream_$i.json > $O/stream_$i.log 2>&1; rc=$?
      python3 -c "import json;d=json.load(open('$O/stream_$i.json'));s=d['sim'];print('calls/s',s['transcriptions_per_s'],'lag p50',s['final_transcript_lag_p50_s'],'batches',d['batch_size_hist'],'conc',d['concurrent_lanes_s'])" ;;
    env:*)
      A=${s#env:}; for kv in ${A//,/ }; do export "$kv"; echo "export $kv"; done; rc=0 ;;
    unenv:*)
      A=${s#unenv:}; for k in ${A//,/ }; do unset "$k"; done; rc=0 ;;
    streamprof)
      export OSW_NO_GRAPH=1
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/sprof_$i -o run -- python3 tools/stream_breakdown.py 32 6.0 $O/stream_prof_$i.json > $O/stream_prof_$i.log 2>&1
      rc=$?; unset OSW_NO_GRAPH
      [ $rc -eq 0 ] && python3 tools/trace_classes.py $O/sprof_$i/run_kernel_trace.csv $O/stream_classes_$i.txt && head -16 $O/stream_classes_$i.txt
      rm -f $O/sprof_$i/run_kernel_trace.csv ;;
    b1)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1prof -o run -- python3 bench.py --steps 1 --warmup 0 --lanes 1 --latency-repeats 4 --latency-warmup 1 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline > $O/b1.json 2> $O/b1.err
      rc=$?; [ $rc -eq 0 ] && python3 tools/b1_breakdown.py $O/b1prof/run_kernel_trace.csv $((5*445)) > $O/b1_breakdown.txt && head -30 $O/b1_breakdown.txt
      rm -f $O/b1prof/run_kernel_trace.csv ;;
    b1beam)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1bprof -o run -- python3 bench.py --steps 1 --warmup 0 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 4 --latency-warmup 1 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline > $O/b1beam.json 2> $O/b1beam.err
      rc=$?; [ $rc -eq 0 ] && python3 tools/b1_breakdown.py $O/b1bprof/run_kernel_trace.csv $((5*445)) > $O/b1beam_breakdown.txt && head -40 $O/b1beam_breakdown.txt
      [ $rc -eq 0 ] && python3 tools/step_timeline.py $O/b1bprof/run_kernel_trace.csv beam_update 1500 > $O/b1beam_step_timeline.txt && cat $O/b1beam_step_timeline.txt
      rm -f $O/b1bprof/run_kernel_trace.csv ;;
    pmcfetch:*)
      # FETCH_SIZE per dispatch of the kernels matching $PMC_MATCH (default gemm8p) over one script
      A=${s#pmcfetch:}; A=${A//,/ }
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$i -o run -- python3 -u $A > $O/pf_$i.log 2>&1; rc=$?
      CSV=$(find $O/pf_$i -name '*counter_collection.csv' | head -1)
      [ -n "$CSV" ] && python3 tools/pmc_dispatch.py $CSV FETCH_SIZE ${PMC_MATCH:-gemm8p} > $O/pmcfetch_$i.txt
      find $O/pf_$i -name '*.csv' -delete
      [ $rc -eq 0 ] && head -40 $O/pmcfetch_$i.txt ;;
    pmcenc)
      # the same SQ counter passes over one 64-window greedy step (one lane)
      for f in 1 2; do
        CN=$(sed -e 's/^pmc: *//' tools/pmc_sq$f.txt)
        timeout -s KILL 300 rocprofv3 --pmc $CN --output-format csv -d $O/pe$f -o run -- python3 bench.py --steps 1 --warmup 0 --lanes 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline > $O/pe$f.log 2>&1; rc=$?
        CSV=$(find $O/pe$f -name '*counter_collection.csv' | head -1)
        [ -n "$CSV" ] && python3 tools/pmc_generic.py $CSV > $O/pmc_enc_$f.txt
        find $O/pe$f -name '*.csv' -delete
        [ $rc -ne 0 ] && break
      done
      [ $rc -eq 0 ] && grep -A1 "enc_attn\|gemm8p" $O/pmc_enc_*.txt | head -40 ;;
    pmcb1beam)
      for f in 1 2; do
        CN=$(sed -e 's/^pmc: *//' tools/pmc_sq$f.txt)
        timeout -s KILL 240 rocprofv3 --pmc $CN --output-format csv -d $O/pq$f -o run -- python3 bench.py --steps 1 --warmup 0 --lanes 1 --batch 4 --latency-repeats 0 --beam5-latency-repeats 1 --latency-warmup 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --rest-callers 0 --no-cpu-baseline > $O/pq$f.log 2>&1; rc=$?
        CSV=$(find $O/pq$f -name '*counter_collection.csv' | head -1)
        [ -n "$CSV" ] && python3 tools/pmc_generic.py $CSV > $O/pmc_b1beam_$f.txt
        find $O/pq$f -name '*.csv' -delete
        [ $rc -ne 0 ] && break
      done
      [ $rc -eq 0 ] && grep -A1 "beam_update\|select_kernel" $O/pmc_b1beam_*.txt | head -20 ;;
    repro)
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/repro -o run -- ./tools/graph_prof_repro 3 300 2 > $O/repro.log 2>&1
      rc=$?; tail -3 $O/repro.log; rm -f $O/repro/run_kernel_trace.csv ;;
    bench:*)
      A=${s#bench:}; A=${A//,/ }
      timeout -k 10 600 python -u bench.py $A > $O/bench_$i.json 2> $O/bench_$i.err; rc=$?
      head -c 600 $O/bench_$i.json; echo ;;
    rprof:*)
      A=${s#rprof:}; A=${A//,/ }
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rprof_$i -o run -- python3 -u $A > $O/rprof_$i.txt 2>&1; rc=$?
      tail -8 $O/rprof_$i.txt
      [ $rc -eq 0 ] && python3 tools/kstats.py $O/rprof_$i/run_kernel_stats.csv 25 > $O/rprof_$i.summary.txt
      rm -f $O/rprof_$i/run_kernel_trace.csv ;;
    py:*)
      A=${s#py:}; A=${A//,/ }
      timeout -k 10 600 python3 -u $A > $O/py_$i.txt 2>&1; rc=$?
      tail -30 $O/py_$i.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then echo "step $s rc $rc: stop"; exit $rc; fi
done
echo "all steps done ($(date +%T))"
