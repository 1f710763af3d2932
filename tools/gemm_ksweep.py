#!/usr/bin/env python3
"""Per-tile overhead of the encoder GEMM: time C = A.W^T (fp32 out, debug entry) at fixed
M x N over K; t(K) = fixed + K * per_k separates the per-tile prologue/epilogue from the
main loop.  usage: gemm_ksweep.py [variant] [M] [N]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

v = int(sys.argv[1]) if len(sys.argv) > 1 else 4
M = int(sys.argv[2]) if len(sys.argv) > 2 else 96000
N = int(sys.argv[3]) if len(sys.argv) > 3 else 5120
d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128, n_text_head=2,
                  n_text_layer=1)
eng = WhisperEngine(d, device=0, max_batch=1)
rng = np.random.default_rng(0)
tiles = ((M + 255) // 256) * ((N + 255) // 256)
rounds = -(-tiles // 256)
for K in [int(k) for k in os.environ.get("KS", "640,1280,2560,5120").split(",")]:
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
    _, ms = eng.debug_gemm(A, W, v, iters=5)
    print(f"variant {v} M={M} N={N} K={K}: {ms * 1e3:.1f} us, {2 * M * N * K / ms / 1e9:.0f} TFLOP/s, "
          f"{ms * 1e3 / rounds:.2f} us per tile round ({tiles} tiles, {rounds} rounds)", flush=True)
