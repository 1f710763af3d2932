#!/usr/bin/env python3
"""Phase times of beam_update (diagnostic library built with -DOSW_STAMPS, loaded through
OSW_LIB): one batch-1 beam-5 decode of a 30 s clip, then the stamps of the last launch's
workgroup 0 (s_memtime ticks = shader cycles; read the shares, not the totals: the stamps'
waits forbid overlaps).  usage: OSW_LIB=.../libosw_stamps.so stamps_probe.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import _lib, synth  # noqa: E402
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd.engine import DecodeConfig, WhisperEngine  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

eng = WhisperEngine(D.LARGE_V3_TURBO, device=0, max_batch=1)
eng.init_random(seed=0)
sup = get_suppressed_tokens(WhisperTokenizer(51866), [-1])
names = ["entry", "state loaded", "loads in LDS", "rows combined", "wave pops", "pops barrier",
         "ranking", "finish bookkeeping", "write-back", "kernel tail"]
N = len(names)
lib = _lib.load()
fn = lib.osw_debug_stamps
fn.argtypes = [C.POINTER(C.c_ulonglong)]
for budget in (40, 200, 400):
    cfg = DecodeConfig(suppress_tokens=sup, beam_size=5, max_length=448, token_budget=(budget,))
    eng.transcribe_batch([synth.chirp_clip(1, 30.0)], cfg)
    buf = (C.c_ulonglong * 32)()
    assert fn(buf) == 0
    t = np.array(buf[:N], dtype=np.int64)
    d = np.diff(t)
    print(f"budget {budget}: total {t[N - 1] - t[0]} cycles; "
          + ", ".join(f"{names[i + 1]} +{d[i]}" for i in range(N - 1)))
eng.close()
