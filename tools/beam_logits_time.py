#!/usr/bin/env python3
"""The beam logits GEMM (M hi/lo rows x the 51866 vocabulary x 1280): the wide 64 x 256 kernel
(debug variant 21) against the beam-rows kernel (20), HIP-event mean of 20 launches."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path
osw_path.load()
import numpy as np
from open_speech_amd import dims as D
from open_speech_amd.engine import WhisperEngine
d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128, n_text_head=2, n_text_layer=1)
eng = WhisperEngine(d, device=0, max_batch=1)
rng = np.random.default_rng(0)
for M in (320, 160, 100):
    A = rng.uniform(-1, 1, (M, 1280)).astype(np.float16)
    W = rng.uniform(-1, 1, (51866, 1280)).astype(np.float16)
    for v in (21, 20):
        C, ms = eng.debug_gemm(A, W, v, iters=20)
        print(json.dumps({"M": M, "variant": v, "us": round(ms * 1e3, 1)}), flush=True)
eng.close()
