# round-4: headline with the shared encoder GEMM grid at 192 (default) / 224 / 256 workgroups, interleaved
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_z; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 12 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --realistic-steps 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for gr in 192 224 256; do
    OSW_GEMM_GRID=$gr timeout -k 10 300 python -u bench.py $A > $O/g${gr}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/g${gr}_$r.json'));print('grid $gr run$r',d['value'],d['ms_per_step'])"
  done
done
