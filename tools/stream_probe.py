#!/usr/bin/env python3
"""Latency of the short calls config 5 (streaming) makes: one utterance prefix of 1-6 s,
json, temperature 0, beam 5, 4 tokens/s length control (random weights), through the
drop-in backend; sequential, then 4 concurrent callers (the reference's streaming
executor width), then with the engine's stage profile.  usage: stream_probe.py [reps]"""
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

R = int(sys.argv[1]) if len(sys.argv) > 1 else 10
SEQ_ONLY = "--sequential-only" in sys.argv
MID = "random:large-v3-turbo"
be = HipWhisperBackend(length_control=4.0)
be.load_model(MID)
if os.environ.get("STREAM_PROBE_MAPS"):   # shared-object map, to attribute a native crash's frames
    with open("/proc/self/maps") as src, open(os.environ["STREAM_PROBE_MAPS"], "w") as dst:
        dst.write(src.read())
wavs = {s: pcm_to_wav(synth.chirp_clip(500, s).tobytes(), 16000) for s in (1.0, 3.0, 6.0)}


def call(w):
    t = time.perf_counter()
    be.transcribe(audio=w, model=MID, language=None, response_format="json", temperature=0.0)
    return (time.perf_counter() - t) * 1e3


for s, w in wavs.items():
    call(w)
    lat = [call(w) for _ in range(R)]
    print(f"sequential {s:.0f} s: p50 {np.median(lat):.1f} ms min {min(lat):.1f}")
if SEQ_ONLY:
    be.unload_model(MID)
    sys.exit(0)
lat = []
lock = threading.Lock()


def worker():
    for _ in range(R):
        v = call(wavs[3.0])
        with lock:
            lat.append(v)


ts = [threading.Thread(target=worker) for _ in range(4)]
t0 = time.perf_counter()
for t in ts:
    t.start()
for t in ts:
    t.join()
wall = time.perf_counter() - t0
print(f"4 concurrent callers, 3 s: p50 {np.median(lat):.1f} ms, {len(lat) / wall:.1f} calls/s")
eng = be._models[MID].engines[0]
eng.set_profiling(True)
call(wavs[3.0])
print({k: round(v, 3) if isinstance(v, float) else v for k, v in eng.profile().items()})
eng.set_profiling(False)
be.unload_model(MID)
