for b in 0 1 2 4 8 32; do
  export OSW_GEMM_BAND=$b
  echo "band $b"
  timeout -k 10 120 python tools/gemm_bench.py sq8 || exit 1
  timeout -k 10 120 python tools/gemm_bench.py enc_fc1 || exit 1
done
