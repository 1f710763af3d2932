# round-4: realistic lengths (row refill) with the shared encoder GEMM grid at 192 (default) / 224 / 256 workgroups
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04_y; mkdir -p $O
export TMPDIR=/tmp
set -e
A="--steps 3 --warmup 1 --latency-repeats 0 --beam5-latency-repeats 0 --beam5 0 --no-cpu-baseline --stream-sessions 0"
for r in 1 2; do
  for gr in 192 224 256; do
    OSW_GEMM_GRID=$gr timeout -k 10 400 python -u bench.py $A > $O/g${gr}_$r.json 2> $O/h.err
    python3 -c "import json;d=json.load(open('$O/g${gr}_$r.json'));x=d['realistic_lengths'];print('grid $gr run$r',x['value'],x['no_refill']['value'])"
  done
done
