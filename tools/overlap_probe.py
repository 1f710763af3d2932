#!/usr/bin/env python3
"""Probe: does running two independent contexts on ONE GPU (two HIP streams, two host
threads) overlap one batch's MFMA-bound encoder with the other's latency/HBM-bound
decoder?  Prints audio-s/s for 1 context vs 2 concurrent contexts.

usage: python tools/overlap_probe.py [batch] [batches_per_ctx] [beam]
"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import osw_path  # noqa: E402

osw_path.load()
import torch  # noqa: E402

from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.engine import DecodeConfig, WhisperEngine  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 3
BEAM = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dims = D.PRESETS["large-v3-turbo"]
torch.cuda.set_device(0)
base = [synth.chirp_clip(i, 30.0) for i in range(8)]
pcm = torch.from_numpy(np.stack([base[i % 8] for i in range(B)])).cuda()
offs = np.arange(B + 1, dtype=np.int64) * 480000
sup = get_suppressed_tokens(WhisperTokenizer(dims.n_vocab), [-1])
cfg = DecodeConfig(suppress_tokens=sup, beam_size=BEAM)
engs = []
for k in range(2):
    e = WhisperEngine(dims, device=0, max_batch=B)
    e.init_random(seed=0)
    engs.append(e)


def run(e, n):
    for _ in range(n):
        e.transcribe_batch(None, cfg, device_pcm=pcm.data_ptr(), offsets=offs)


for e in engs:
    run(e, 1)  # warm-up (graph capture)
torch.cuda.synchronize()
t = time.perf_counter()
run(engs[0], NB)
t1 = time.perf_counter() - t
print(f"1 ctx  B={B} beam={BEAM}: {NB} batches in {t1:.3f}s -> {NB * B * 30 / t1:.1f} audio-s/s", flush=True)
th = [threading.Thread(target=run, args=(e, NB)) for e in engs]
t = time.perf_counter()
for x in th:
    x.start()
for x in th:
    x.join()
t2 = time.perf_counter() - t
print(f"2 ctx  B={B} beam={BEAM}: {2 * NB} batches in {t2:.3f}s -> {2 * NB * B * 30 / t2:.1f} audio-s/s "
      f"({t1 * 2 / t2:.2f}x)", flush=True)
for e in engs:
    e.close()
