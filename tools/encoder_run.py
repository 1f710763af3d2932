#!/usr/bin/env python3
"""Driver for PMC counter passes: log-mel + encoder + cross-K/V of 64 x 30 s clips
(large-v3-turbo, random weights), run --iters times; with --decode-steps N also N
greedy decoder steps per iteration, launched eagerly (no hipGraph) so every decoder
kernel dispatch is attributed."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.engine import DecodeConfig, WhisperEngine  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=1)
ap.add_argument("--decode-steps", type=int, default=0)
a = ap.parse_args()
eng = WhisperEngine(D.LARGE_V3_TURBO, device=0, max_batch=a.batch)
eng.init_random(seed=0)
clips = [synth.chirp_clip(i % 8, 30.0) for i in range(a.batch)]
if a.decode_steps:
    eng.set_profiling(True, eager_decode=True)
    cfg = DecodeConfig(suppress_tokens=get_suppressed_tokens(WhisperTokenizer(D.LARGE_V3_TURBO.n_vocab), [-1]),
                       max_length=3 + a.decode_steps)
for _ in range(a.iters):
    nf = eng.log_mel(clips)
    eng.encode([(i, 0, min(3000, nf[i] - 1)) for i in range(a.batch)])
    if a.decode_steps:
        eng.decode(a.batch, cfg)
eng.close()
print("ok")
