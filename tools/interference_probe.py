#!/usr/bin/env python3
"""Which stage of a second context disturbs a decoding context?  Context B transcribes
the same two clips repeatedly while context A loops one stage (mel / encoder /
decoder) on its own stream; B's sum_logprob must stay bit-identical."""
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
from open_speech_amd.engine import DecodeConfig, WhisperEngine  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

d = D.TINY_TEST
w = weights.random_weights(d, seed=1234, emb_std=0.5)
A = WhisperEngine(d, device=0, max_batch=4)
A.load_weights(w)
B = A.sibling(max_batch=4)
sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
cfg = DecodeConfig(suppress_tokens=sup, max_length=64)
clips = [synth.chirp_clip(31, 30.0), synth.chirp_clip(32, 11.0)]
wins = [(0, 0, 3000), (1, 0, 1099)]


def sig(outs):
    return tuple(round(o.sum_logprob, 7) for o in outs)


ref = sig(B.transcribe_batch(clips, cfg))
A.transcribe_batch(clips, cfg)
stages = {
    "mel": lambda: A.log_mel(clips),
    "encode": lambda: A.encode(wins),
    "decode": lambda: A.decode(2, cfg),
    "all": lambda: A.transcribe_batch(clips, cfg),
}
_rng = np.random.default_rng(0)
_ga = (_rng.standard_normal((3000, 1280)) * 0.1).astype(np.float16)
_gw = (_rng.standard_normal((1280, 1280)) * 0.1).astype(np.float16)
_ge = (_rng.standard_normal((1500, d.n_audio_state))).astype(np.float32)
for _v in (1, 2, 4):
    stages[f"gemm{_v}"] = (lambda v=_v: A.debug_gemm(_ga, _gw, variant=v, iters=20))
stages["layer"] = lambda: A.encoder_layer(0, _ge)
for name in sys.argv[1:] or list(stages):
    stop = []

    def loop(fn=stages[name]):
        while not stop:
            fn()

    t = threading.Thread(target=loop)
    t.start()
    bad = 0
    for _ in range(8):
        if sig(B.transcribe_batch(clips, cfg)) != ref:
            bad += 1
    stop.append(1)
    t.join()
    A.log_mel(clips)
    A.encode(wins)
    print(f"A loops {name}: {bad}/8 of B's calls drifted", flush=True)
B.close()
A.close()
