#!/usr/bin/env python3
"""Run-to-run determinism probe on the tiny test model: the same two clips through
one engine several times, then through a sibling, then through both concurrently.
Prints sum_logprob per call so a drift can be attributed to a context or to
concurrency."""
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
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 4
eng = WhisperEngine(d, device=0, max_batch=mb)
eng.load_weights(weights.random_weights(d, seed=1234, emb_std=0.5))
sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
cfg = DecodeConfig(suppress_tokens=sup, max_length=64)
clips = [synth.chirp_clip(31, 30.0), synth.chirp_clip(32, 11.0)]


def sig(outs):
    return tuple((len(o.tokens), round(o.sum_logprob, 7)) for o in outs)


print("parent seq:", [sig(eng.transcribe_batch(clips, cfg)) for _ in range(4)])
print("parent single:", [sig(eng.transcribe_batch(clips[:1], cfg)) for _ in range(2)])
sib = eng.sibling(max_batch=2)
print("sibling seq:", [sig(sib.transcribe_batch(clips, cfg)) for _ in range(4)])
got = {}


def run(name, e):
    got[name] = [sig(e.transcribe_batch(clips, cfg)) for _ in range(3)]


th = [threading.Thread(target=run, args=(n, e)) for n, e in (("a", eng), ("b", sib))]
for t in th:
    t.start()
for t in th:
    t.join()
print("concurrent:", got)
wts = weights.random_weights(d, seed=1234, emb_std=0.5)
bad = []
for name, arr in wts.items():
    if name == "enc.conv1.w":
        continue
    got_w = eng.get_weight(name)
    want = np.asarray(arr, dtype=got_w.dtype).ravel()
    if not np.array_equal(got_w, want):
        bad.append((name, int((got_w != want).sum())))
print("weights changed:", bad)
# two independent contexts (own weight copies) side by side
eng2 = WhisperEngine(d, device=0, max_batch=mb)
eng2.load_weights(weights.random_weights(d, seed=1234, emb_std=0.5))
got = {}
th = [threading.Thread(target=run, args=(n, e)) for n, e in (("a", eng), ("c", eng2))]
for t in th:
    t.start()
for t in th:
    t.join()
print("independent:", got)
eng2.close()
# the sibling next to unrelated GPU work on another stream
stop = []


def noise():
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    x = torch.randn(4096, 4096, device="cuda", dtype=torch.float16)
    with torch.cuda.stream(s):
        while not stop:
            for _ in range(20):
                x = (x @ x).clamp_(-1, 1)
            s.synchronize()


for rep in range(3):
    got = {}
    stop.clear()
    tn = threading.Thread(target=noise)
    tn.start()
    run("b", sib)
    run("a", eng)
    stop.append(1)
    tn.join()
    print("noise:", got)
sib.close()
eng.close()
