#!/usr/bin/env python3
"""Encoder time (log-mel + conv stem + 32 layers + cross-K/V, HIP events) of 1-4 windows of
large-v3-turbo, the shapes of streaming calls and session admissions.  The tile policy is
read from the environment (OSW_GEMM_HALF=0/1), so run it once per setting.
usage: small_encoder_time.py [windows ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

wins = [int(x) for x in sys.argv[1:]] or [1, 2, 3, 4]
eng = WhisperEngine(D.LARGE_V3_TURBO, device=0, max_batch=max(wins))
eng.init_random(seed=0)
clips = [synth.chirp_clip(i, 30.0) for i in range(max(wins))]
nf = eng.log_mel(clips)
eng.set_profiling(True)
out = {"OSW_GEMM_HALF": os.environ.get("OSW_GEMM_HALF", "default")}
for w in wins:
    win = [(i, 0, min(3000, nf[i] - 1)) for i in range(w)]
    for _ in range(3):
        eng.encode(win)
    ts, parts = [], []
    for _ in range(10):
        eng.set_profiling(True)  # resets the accumulated timers
        eng.encode(win)
        p = eng.profile()
        ts.append(p["encoder_ms"] + p["crosskv_ms"])
        parts.append((p["enc_gemm_ms"], p["enc_attn_ms"]))
    i = sorted(range(len(ts)), key=ts.__getitem__)[len(ts) // 2]
    out[f"w{w}_ms"] = round(ts[i], 3)
    out[f"w{w}_gemm_attn_ms"] = [round(parts[i][0], 3), round(parts[i][1], 3)]
print(json.dumps(out), flush=True)
eng.close()
