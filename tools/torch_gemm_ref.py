#!/usr/bin/env python3
"""Reference point for the encoder GEMM shapes: torch.matmul (hipBLASLt / rocBLAS) fp16
with fp32 accumulation on the same M x N x K as gemm8p_kernel, timed with HIP events."""
import torch

torch.backends.cuda.matmul.allow_fp16_reduced_precision_reduction = False
SHAPES = [("enc_qkv", 96000, 3840, 1280), ("enc_o", 96000, 1280, 1280), ("enc_fc1", 96000, 5120, 1280),
          ("enc_fc2", 96000, 1280, 5120), ("sq8192", 8192, 8192, 8192)]
for name, M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16)
    for _ in range(3):
        c = a @ w.t()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 10
    e0.record()
    for _ in range(it):
        c = a @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"{name}: M={M} N={N} K={K} {ms * 1e3:.1f} us {2 * M * N * K / ms / 1e9:.1f} TFLOP/s", flush=True)
