#!/usr/bin/env python3
"""Time the GEMM variants on the encoder / decoder shapes (GPU).

usage: gemm_bench.py [shape-prefix] [variants]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

SHAPES = [  # name, M, N, K, variants
    ("sq4096", 4096, 4096, 4096, (2, 4)), ("sq8192", 8192, 8192, 8192, (2, 4)),
    ("enc_qkv", 96000, 3840, 1280, (1, 2, 4)), ("enc_o", 96000, 1280, 1280, (1, 2, 4)),
    ("enc_fc1", 96000, 5120, 1280, (1, 2, 4)), ("enc_fc2", 96000, 1280, 5120, (1, 2, 4)),
    ("dec_qkv", 64, 3840, 1280, (3,)), ("dec_fc2", 64, 1280, 5120, (3,)), ("dec_o", 64, 1280, 1280, (3,)),
    ("dec_qkv16", 16, 3840, 1280, (3,)), ("dec_logits", 64, 51866, 1280, (3, 1)), ("dec_logits32", 32, 51866, 1280, (3, 1)),
    ("dec_logits16", 16, 51866, 1280, (3,)),
    ("dec_logits_b1", 1, 51866, 1280, (3,)), ("dec_fc1_b1", 1, 5120, 1280, (3,)),
]
d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128, n_text_head=2,
                  n_text_layer=1)
eng = WhisperEngine(d, device=0, max_batch=1)
rng = np.random.default_rng(0)
out = []
only = sys.argv[1] if len(sys.argv) > 1 else ""
# optional comma (or colon) list of variants overriding each shape's own (e.g. 9,8,10,4: the 8-phase
# kernel with no epilogue / fp16 out / GELU fp16 out / fp32 out)
force = tuple(int(v) for v in sys.argv[2].replace(":", ",").split(",")) if len(sys.argv) > 2 else None
for name, M, N, K, vs in SHAPES:
    if only and not name.startswith(only):
        continue
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
    first = None
    for v in force or vs:
        C, ms = eng.debug_gemm(A, W, v, iters=5)
        if first is None:
            first = C
        same = bool(np.array_equal(C.view(np.uint32), first.view(np.uint32)))
        tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
        gbs = (N * K * 2 + M * K * 2 + M * N * 4) / (ms * 1e-3) / 1e9
        r = {"shape": name, "M": M, "N": N, "K": K, "variant": v, "ms": round(ms, 4), "TFLOPs": round(tf, 1),
             "GBs": round(gbs, 1), "bits_equal_first": same}
        out.append(r)
        print(json.dumps(r), flush=True)
eng.close()
