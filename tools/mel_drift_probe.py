#!/usr/bin/env python3
"""Does the log-mel kernel give bit-identical output while another context's encoder runs?
Context B computes the log-mel of two clips repeatedly (get_mel: the normalised fp32
values) while context A loops a stage on its own stream; every B result is compared
element-wise with B's lone result.  Reports, per stage, how many calls differed, how many
elements, the largest difference and the frames it touched.  OSW_LIB selects the library
build (tools/gpu_pk_bisect.sh)."""
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
import torch  # noqa: E402

torch.cuda.set_device(0)
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth, weights  # noqa: E402
from open_speech_amd.engine import WhisperEngine  # noqa: E402

d = D.TINY_TEST
w = weights.random_weights(d, seed=1234, emb_std=0.5)
A = WhisperEngine(d, device=0, max_batch=4)
A.load_weights(w)
B = A.sibling(max_batch=4)
clips = [synth.chirp_clip(31, 30.0), synth.chirp_clip(32, 11.0)]
wins = [(0, 0, 3000), (1, 0, 1099)]
calls = int(os.environ.get("PROBE_CALLS", "16"))


def mels(e):
    e.log_mel(clips)
    return [e.get_mel(i).copy() for i in range(len(clips))]


ref = mels(B)
A.log_mel(clips)
A.encode(wins)
_ge = (np.random.default_rng(0).standard_normal((1500, d.n_audio_state))).astype(np.float32)
stages = {
    "none": None,
    "encode": lambda: A.encode(wins),
    "layer": lambda: A.encoder_layer(0, _ge),
}
for name in sys.argv[1:] or list(stages):
    stop = []
    fn = stages[name]

    def loop():
        while not stop:
            fn()

    t = threading.Thread(target=loop) if fn else None
    if t:
        t.start()
    bad, n_el, worst, frames = 0, 0, 0.0, set()
    for _ in range(calls):
        got = mels(B)
        diff = False
        for g, r in zip(got, ref):
            ne = g != r
            if ne.any():
                diff = True
                n_el += int(ne.sum())
                worst = max(worst, float(np.abs(g - r).max()))
                frames.update(np.nonzero(ne.any(axis=0))[0][:32].tolist())
        bad += diff
    stop.append(1)
    if t:
        t.join()
    print(f"A loops {name}: {bad}/{calls} mel calls differed, {n_el} elements, max |diff| {worst:.3g}, "
          f"frames {sorted(frames)[:24]}", flush=True)
B.close()
A.close()
