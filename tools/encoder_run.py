#!/usr/bin/env python3
"""Encoder-only driver for PMC counter passes: log-mel + encoder + cross-K/V of
64 x 30 s clips (large-v3-turbo, random weights), run --iters times."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=1)
a = ap.parse_args()
eng = WhisperEngine(D.LARGE_V3_TURBO, device=0, max_batch=a.batch)
eng.init_random(seed=0)
clips = [synth.chirp_clip(i % 8, 30.0) for i in range(a.batch)]
for _ in range(a.iters):
    nf = eng.log_mel(clips)
    eng.encode([(i, 0, min(3000, nf[i] - 1)) for i in range(a.batch)])
eng.close()
print("ok")
