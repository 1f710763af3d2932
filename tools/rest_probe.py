#!/usr/bin/env python3
"""REST-style load on the drop-in backend (the batcher's STT_HIP_BATCH_GAP_MS
was measured only for streaming): C concurrent callers, each posting R 30 s WAVs (json,
language None, the backend's default decoding) with exponentially jittered think time
(mean J ms) between calls.  Prints calls/s and latency percentiles for the gap setting in
the environment.  usage: rest_probe.py [callers=16] [calls_per_caller=6] [jitter_ms=40]"""
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
os.environ.setdefault("STT_HIP_TOKENS_PER_SEC", "4")
be = HipWhisperBackend()
be.load_model(MID)
wavs = [pcm_to_wav(synth.chirp_clip(800 + i, 30.0).tobytes(), 16000) for i in range(8)]
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
print(f"gap_ms {gap}: {C} callers x {R} calls, jitter {J:.0f} ms: {len(lat) / wall:.2f} calls/s, "
      f"latency p50 {np.median(lat):.0f} ms p95 {np.percentile(lat, 95):.0f} ms", flush=True)
be.unload_model(MID)
