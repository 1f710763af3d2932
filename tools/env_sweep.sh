# headline bench under A/B environment switches (exploration)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-envsweep}; mkdir -p $O
timeout -k 10 240 python -u bench.py --steps 6 --beam5 0 --latency-repeats 1 --no-cpu-baseline > $O/base.json 2> $O/base.err
OSW_GEMM128=1 timeout -k 10 240 python -u bench.py --steps 6 --beam5 0 --latency-repeats 1 --no-cpu-baseline > $O/g128.json 2> $O/g128.err
OSW_GEMM_2PHASE=1 timeout -k 10 240 python -u bench.py --steps 6 --beam5 0 --latency-repeats 1 --no-cpu-baseline > $O/g2p.json 2> $O/g2p.err
OSW_GEMM128=1 timeout -k 10 240 python -u bench.py --steps 6 --beam5 0 --latency-repeats 1 --no-cpu-baseline --lanes 4 > $O/g128_l4.json 2> $O/g128_l4.err
