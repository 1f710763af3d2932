#!/usr/bin/env python3
"""REST-style load on the drop-in backend (the batcher's STT_HIP_BATCH_GAP_MS
was measured only for streaming): C concurrent callers, each posting R 30 s WAVs (json,
language None, the backend's default decoding) with exponentially jittered think time
(mean J ms) between calls.  Prints calls/s and latency percentiles for the gap setting in
the environment.  ``mix``: clips of 4-75 s instead (1-3 windows each, windows of different
lengths and token budgets), the load continuous batching (STT_HIP_CONTINUOUS=1) is for.
usage: rest_probe.py [callers=16] [calls_per_caller=6] [jitter_ms=40] [mix]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.audio import pcm_to_wav  # noqa: E402
from open_speech_amd.backend import HipWhisperBackend  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 16
R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
J = float(sys.argv[3]) if len(sys.argv) > 3 else 40.0
MID = "random:large-v3-turbo"
be = HipWhisperBackend(length_control=4.0)
be.load_model(MID)
MIX = len(sys.argv) > 4 and sys.argv[4] == "mix"
LENS = (4.0, 12.0, 30.0, 45.0, 75.0, 20.0, 8.0, 60.0) if MIX else (30.0,) * 8
wavs = [pcm_to_wav(synth.chirp_clip(800 + i, s).tobytes(), 16000) for i, s in enumerate(LENS)]
be.transcribe(audio=wavs[0], model=MID, language=None, response_format="json")  # warm (graphs)
lat, lock = [], threading.Lock()


def caller(i):
    rng = np.random.default_rng(i)
    for k in range(R):
        time.sleep(rng.exponential(J / 1000.0))
        t = time.perf_counter()
        be.transcribe(audio=wavs[(i + k) % len(wavs)], model=MID, language=None, response_format="json")
        with lock:
            lat.append((time.perf_counter() - t) * 1e3)


ts = [threading.Thread(target=caller, args=(i,)) for i in range(C)]
t0 = time.perf_counter()
for t in ts:
    t.start()
for t in ts:
    t.join()
wall = time.perf_counter() - t0
gap = os.environ.get("STT_HIP_BATCH_GAP_MS", "1 (default)")
mode = "continuous" if os.environ.get("STT_HIP_CONTINUOUS", "1") != "0" else "batch"
print(f"{mode}{' mix' if MIX else ''} audio {sum(LENS[(i + k) % 8] for i in range(C) for k in range(R)) / wall:.0f} s/s, "
      f"gap_ms {gap}: {C} callers x {R} calls, jitter {J:.0f} ms: {len(lat) / wall:.2f} calls/s, "
      f"latency p50 {np.median(lat):.0f} ms p95 {np.percentile(lat, 95):.0f} ms", flush=True)
be.unload_model(MID)
