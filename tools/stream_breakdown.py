#!/usr/bin/env python3
"""Where a config-5 call's time goes (BASELINE configs[4], bench.stream_sessions).

Runs the streaming simulation of bench.py (n sessions, 100 ms chunks, 4-thread
executor, beam 5) with wall-clock instrumentation of the runner and the engine:
every batch a lane runs (size, start, end), and inside it the engine's log_mel /
encode (enqueue only) / decode (synchronous: waits for the encoder too) calls.
Prints a JSON summary: batch-size histogram, per-lane busy fraction, the time a
call spends queued before its batch starts, and per batch size the median wall
time of each engine stage plus the host time outside them (Python seek loop,
WAV parse, tokenizer, futures).

usage: stream_breakdown.py [sessions] [speech_s] [out.json]
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
from open_speech_amd import runner as R  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

n_sess = int(sys.argv[1]) if len(sys.argv) > 1 else 32
speech = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
out_path = sys.argv[3] if len(sys.argv) > 3 else None

lock = threading.Lock()
batches = []                      # (lane, n, t0, t1, [queued_s per request], stages{})
tls = threading.local()


def wrap_engine(name):
    orig = getattr(WhisperEngine, name)

    def f(self, *a, **k):
        t = time.perf_counter()
        try:
            return orig(self, *a, **k)
        finally:
            st = getattr(tls, "stages", None)
            if st is not None:
                st[name] = st.get(name, 0.0) + time.perf_counter() - t
                if name == "decode":
                    st["decode_calls"] = st.get("decode_calls", 0) + 1
    setattr(WhisperEngine, name, f)


for nm in ("log_mel", "encode", "decode"):
    wrap_engine(nm)

orig_submit = R.BatchRunner.submit_req


def submit_req(self, r, *a, **k):
    if not hasattr(r, "_t_sub"):
        r._t_sub = time.perf_counter()
    return orig_submit(self, r, *a, **k)


R.BatchRunner.submit_req = submit_req
orig_run = R._Worker._run_batch


def run_batch(self, batch):
    tls.stages = {}
    t0 = time.perf_counter()
    try:
        return orig_run(self, batch)
    finally:
        t1 = time.perf_counter()
        with lock:
            batches.append((self.idx, len(batch), t0, t1, [t0 - getattr(r, "_t_sub", t0) for r in batch],
                            dict(tls.stages)))
        tls.stages = None


R._Worker._run_batch = run_batch

res = bench.stream_sessions(n_sess, speech)
wall = res["wall_s"]
by_n = defaultdict(list)
for b in batches:
    by_n[b[1]].append(b)
lanes = defaultdict(float)
for b in batches:
    lanes[b[0]] += b[3] - b[2]
# overlap: how much of the wall time had >= 2 lanes busy
ev = sorted([(b[2], 1) for b in batches] + [(b[3], -1) for b in batches])
busy = defaultdict(float)
cur, last = 0, ev[0][0] if ev else 0.0
for t, d in ev:
    busy[cur] += t - last
    cur += d
    last = t
summary = {
    "sim": res,
    "batches": len(batches),
    "batch_size_hist": {int(k): len(v) for k, v in sorted(by_n.items())},
    "lane_busy_s": {int(k): round(v, 3) for k, v in sorted(lanes.items())},
    "concurrent_lanes_s": {int(k): round(v, 3) for k, v in sorted(busy.items())},
    "queued_before_batch_ms_p50": round(1e3 * float(np.median([q for b in batches for q in b[4]])), 2),
    "per_batch_size": {},
}
for n, bs in sorted(by_n.items()):
    wall_ms = [1e3 * (b[3] - b[2]) for b in bs]
    st = {k: [1e3 * b[5].get(k, 0.0) for b in bs] for k in ("log_mel", "encode", "decode")}
    host = [w - sum(st[k][i] for k in st) for i, w in enumerate(wall_ms)]
    summary["per_batch_size"][int(n)] = {
        "count": len(bs), "batch_wall_ms_p50": round(float(np.median(wall_ms)), 2),
        **{f"{k}_ms_p50": round(float(np.median(v)), 2) for k, v in st.items()},
        "host_outside_engine_ms_p50": round(float(np.median(host)), 2),
        "decode_calls_p50": float(np.median([b[5].get("decode_calls", 0) for b in bs])),
    }
txt = json.dumps(summary, indent=1)
print(txt)
if out_path:
    with open(out_path, "w") as fh:
        fh.write(txt)
