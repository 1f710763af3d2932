#!/usr/bin/env python3
"""Encoder GEMM shapes at 1, 2, 4 and 8 windows (M = 1500 w): every tile variant timed
(debug entry, fp32 out) and checked bit-identical against the 128 double-buffered tile.
variants: 1 = 128 tile, 4 = 8-phase 256, 6 = 64 ring, 7 = 64 tile, 11 = 128 ring, 16 = half-width
256 x 128 tile (9 / 17: the 8-phase / half-width main loops alone, not compared).  usage: small_gemm_bench.py [windows] [variants] [gemms]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128, n_text_head=2,
                  n_text_layer=1)
eng = WhisperEngine(d, device=0, max_batch=1)
rng = np.random.default_rng(0)
wins = [int(x) for x in sys.argv[1].replace(":", ",").split(",")] if len(sys.argv) > 1 else [1, 2, 3, 4]
variants = [int(x) for x in sys.argv[2].replace(":", ",").split(",")] if len(sys.argv) > 2 else [1, 6, 7, 11, 4]
gemms = sys.argv[3].replace(":", ",").split(",") if len(sys.argv) > 3 else ["qkv", "o", "fc1", "fc2", "xkv"]
shapes = {"qkv": (3840, 1280), "o": (1280, 1280), "fc1": (5120, 1280), "fc2": (1280, 5120), "xkv": (10240, 1280)}
for w in wins:
    M = 1500 * w
    for name in gemms:
        N, K = shapes[name]
        A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
        W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
        ref = None
        for v in variants:
            C, ms = eng.debug_gemm(A, W, v, iters=20)
            if ref is None:
                ref = C
            same = bool(np.array_equal(C, ref)) if v not in (9, 17) else None
            tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
            print(json.dumps({"windows": w, "gemm": name, "M": M, "N": N, "K": K, "variant": v, "us": round(ms * 1e3, 1),
                              "TFLOPs": round(tf, 1), "bit_identical": same}), flush=True)
eng.close()
