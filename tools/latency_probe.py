#!/usr/bin/env python3
"""Batch-1 latency probe (BASELINE configs[1]): one 30 s clip, repeated; prints the
per-call wall time and the engine's stage split.  Run under rocprofv3 --kernel-trace
to get per-kernel durations and inter-kernel gaps (tools/kstats_db.py --gaps).

usage: python tools/latency_probe.py [repeats] [beam] [batch]
"""
import os
import sys
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

R = int(sys.argv[1]) if len(sys.argv) > 1 else 5
BEAM = int(sys.argv[2]) if len(sys.argv) > 2 else 1
B = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dims = D.PRESETS["large-v3-turbo"]
torch.cuda.set_device(0)
pcm = torch.from_numpy(np.stack([synth.chirp_clip(999 + i, 30.0) for i in range(B)])).cuda()
offs = np.arange(B + 1, dtype=np.int64) * 480000
sup = get_suppressed_tokens(WhisperTokenizer(dims.n_vocab), [-1])
cfg = DecodeConfig(suppress_tokens=sup, beam_size=BEAM)
e = WhisperEngine(dims, device=0, max_batch=max(B, 1))
e.init_random(seed=0)
e.transcribe_batch(None, cfg, device_pcm=pcm.data_ptr(), offsets=offs)
lat = []
for _ in range(R):
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = e.transcribe_batch(None, cfg, device_pcm=pcm.data_ptr(), offsets=offs)
    lat.append((time.perf_counter() - t) * 1e3)
e.set_profiling(True)
e.transcribe_batch(None, cfg, device_pcm=pcm.data_ptr(), offsets=offs)
p = e.profile()
e.set_profiling(False)
print(f"B={B} beam={BEAM}: p50 {np.median(lat):.2f} ms (min {min(lat):.2f}), tokens {len(out[0].tokens)}")
print({k: round(v, 3) if isinstance(v, float) else v for k, v in p.items()})
e.close()
