#!/usr/bin/env python3
"""Where a config-5 call's time goes on the deployed (continuous, decode-session) path.

Runs bench.stream_sessions (n sessions, 100 ms chunks, 4-thread executor, beam 5) with
wall-clock instrumentation of every lane's engine calls: session_add, the admission step
(session_step with max_chunks 0: the windows' log-mel staging and encoder, waited for),
the decode chunks (session_step with max_chunks >= 1: 8 decoder steps each) and
session_begin / session_end, plus the backend's own host work per call
(HipWhisperBackend._run_inference outside runner.transcribe: WAV parse, options, response
shaping).  Prints a JSON summary: per lane the seconds inside each engine call kind and
the lane's host time outside them, and per call the median host time in the backend.

usage: stream_session_breakdown.py [sessions] [speech_s] [out.json]
"""
import json
import os
import sys
import threading
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import osw_path  # noqa: E402

osw_path.load()
import bench  # noqa: E402
from open_speech_amd import backend as B  # noqa: E402
from open_speech_amd import runner as R  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

n_sess = int(sys.argv[1]) if len(sys.argv) > 1 else 32
speech = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
out_path = sys.argv[3] if len(sys.argv) > 3 else None

lock = threading.Lock()
per_thread = defaultdict(lambda: defaultdict(float))     # thread name -> kind -> seconds
counts = defaultdict(lambda: defaultdict(int))


def wrap(name, kind_of):
    orig = getattr(WhisperEngine, name)

    def f(self, *a, **k):
        t = time.perf_counter()
        try:
            return orig(self, *a, **k)
        finally:
            kind = kind_of(a, k)
            th = threading.current_thread().name
            with lock:
                per_thread[th][kind] += time.perf_counter() - t
                counts[th][kind] += 1
    setattr(WhisperEngine, name, f)


wrap("session_add", lambda a, k: "add")
wrap("session_step", lambda a, k: "admit" if (a[0] if a else k.get("max_chunks", 64)) == 0 else "chunk")
wrap("session_begin", lambda a, k: "begin_end")
wrap("session_end", lambda a, k: "begin_end")
wrap("session_release_clip", lambda a, k: "release")

lane_wall = defaultdict(float)
orig_run = R._SessionLane.run


def run(self):
    t = time.perf_counter()
    try:
        return orig_run(self)
    finally:
        lane_wall[self.name] += time.perf_counter() - t


R._SessionLane.run = run

host_ms = []
orig_inf = B.HipWhisperBackend._run_inference
orig_tr = R.BatchRunner.transcribe
tls = threading.local()


def transcribe(self, *a, **k):
    t = time.perf_counter()
    try:
        return orig_tr(self, *a, **k)
    finally:
        tls.in_runner = getattr(tls, "in_runner", 0.0) + time.perf_counter() - t


def run_inference(self, *a, **k):
    tls.in_runner = 0.0
    t = time.perf_counter()
    try:
        return orig_inf(self, *a, **k)
    finally:
        with lock:
            host_ms.append(1e3 * (time.perf_counter() - t - tls.in_runner))


R.BatchRunner.transcribe = transcribe
B.HipWhisperBackend._run_inference = run_inference

res = bench.stream_sessions(n_sess, speech)
wall = res["wall_s"]
lanes = {}
for th, kinds in sorted(per_thread.items()):
    if not th.startswith("osw-lane"):
        continue
    inside = sum(kinds.values())
    lanes[th] = {**{f"{k}_s": round(v, 3) for k, v in sorted(kinds.items())},
                 **{f"{k}_n": counts[th][k] for k in sorted(kinds)},
                 "inside_engine_s": round(inside, 3), "wall_s": round(wall, 3),
                 "chunk_ms_mean": round(1e3 * kinds.get("chunk", 0.0) / max(1, counts[th]["chunk"]), 3),
                 "admit_ms_mean": round(1e3 * kinds.get("admit", 0.0) / max(1, counts[th]["admit"]), 3)}
summary = {"sim": res, "lanes": lanes,
           "backend_host_ms_per_call_p50": round(float(np.median(host_ms)), 3) if host_ms else None,
           "backend_host_ms_per_call_mean": round(float(np.mean(host_ms)), 3) if host_ms else None,
           "calls": len(host_ms)}
txt = json.dumps(summary, indent=1)
print(txt)
if out_path:
    with open(out_path, "w") as fh:
        fh.write(txt)
