# A/B of the encoder baton (OSW_ENC_BATON=0 vs 1), then a kernel trace of the baton run.  usage: gpu_baton_ab.sh OUT
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-baton}; mkdir -p $O
ARGS="--steps 9 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --stream-sessions 0 --no-cpu-baseline"
for r in 1 2; do
  for b in 0 1; do
    OSW_ENC_BATON=$b timeout -k 10 300 python -u bench.py $ARGS > $O/bench_b${b}_$r.json 2> $O/bench_b${b}_$r.err
    python3 -c "import json,sys;d=json.load(open('$O/bench_b${b}_$r.json'));print('baton',$b,'run',$r,d['value'],d['beam5']['value'] if d.get('beam5') else None,d['realistic_lengths']['value'] if d.get('realistic_lengths') else None)"
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 6 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --beam5-steps 0 --realistic-steps 0 --stream-sessions 0 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
gzip -f $O/prof/run_kernel_trace.csv
