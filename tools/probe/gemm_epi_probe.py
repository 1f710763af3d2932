#!/usr/bin/env python3
"""The 8-phase GEMM's epilogue forms (GPU) on the encoder shapes at 64 windows,
interleaved over rounds: debug variants 9 (no epilogue), 8 / 12 (fp16 out, accumulators
transposed / not), 10 / 13 (fp16 + GELU, transposed / not); each transposed form must
equal its plain one bit for bit.  (Round 4 r04_t, an earlier build: 15 / 14 = fp32 out,
transposed / not; the fp32 forms stay plain)  (Round 4 r04_p, an
earlier build: 12 = LDS image without the global stores, 13 = stores without the image.)"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

SHAPES = [("fc1", 96000, 5120, 1280), ("qkv", 96000, 3840, 1280), ("fc2", 96000, 1280, 5120)]
VARIANTS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "9,8,12,10,13").split(",")]
SAME = {12: 8, 13: 10}
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128, n_text_head=2,
                  n_text_layer=1)
eng = WhisperEngine(d, device=0, max_batch=1)
rng = np.random.default_rng(0)
for name, M, N, K in SHAPES:
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
    digest = {}
    for r in range(ROUNDS):
        for v in VARIANTS:
            C, ms = eng.debug_gemm(A, W, v, iters=5)
            rec = {"shape": name, "round": r, "variant": v, "us": round(ms * 1e3, 1),
                   "TFLOPs": round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)}
            if v in (8, 10, 12, 13):
                raw = np.ascontiguousarray(C).view(np.uint16).ravel()
                digest[v] = hashlib.sha1(raw[:M * N].tobytes()).hexdigest()
                if SAME.get(v) in digest:
                    rec["equal_to_%d" % SAME[v]] = digest[v] == digest[SAME[v]]
            print(json.dumps(rec), flush=True)
eng.close()
