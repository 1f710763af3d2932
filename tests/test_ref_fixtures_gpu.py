"""GPU ingest (csrc/ingest.hip through osw_ingest_*) against the REFERENCE's own
outputs (tools/make_ref_fixtures.py ran /root/reference's functions): byte-exact.

* preprocess_stt_audio  /root/reference/src/audio/preprocessing.py:53-63
* resample_pcm16        /root/reference/src/streaming.py:55-91
"""
import hashlib
import json
import os

import numpy as np
import pytest

import ref_inputs
from open_speech_amd import ingest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLD, "ref_fixtures.json")))
ARR = np.load(os.path.join(GOLD, "ref_fixtures.npz"))
PP = {r["name"]: r for r in META["preprocess"]}
RS = {r["name"]: r for r in META["resample"]}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _diff(got: bytes, key: str) -> str:
    if key not in ARR:
        return ""
    want = ARR[key].tobytes()
    a = np.frombuffer(got[44 if key.startswith("pp_") else 0:], np.int16)
    b = np.frombuffer(want[44 if key.startswith("pp_") else 0:], np.int16)
    if a.shape != b.shape:
        return f" shapes {a.shape} vs {b.shape}"
    d = np.nonzero(a != b)[0]
    return f" {d.size} samples differ, first {d[:5].tolist()}: {a[d[:5]].tolist()} vs {b[d[:5]].tolist()}"


@pytest.mark.parametrize("name,wav", list(ref_inputs.preprocess_cases()), ids=lambda v: v if isinstance(v, str) else "")
def test_gpu_preprocess_matches_reference(name, wav):
    rec = PP[name]
    out = ingest.preprocess_stt_audio(wav, noise_reduce=False, normalize=True)
    assert len(out) == rec["out_len"], name
    assert sha(out) == rec["out_sha256"], name + _diff(out, "pp_" + name)


@pytest.mark.parametrize("case", list(ref_inputs.resample_cases()), ids=lambda c: c[0])
def test_gpu_resample_matches_reference(case):
    name, pcm, fr, to = case
    rec = RS[name]
    out = ingest.resample_pcm16(pcm, fr, to)
    assert len(out) == rec["out_len"], name
    assert sha(out) == rec["out_sha256"], name + _diff(out, "rs_" + name)


def test_gpu_mean_square_is_numpy_reduction():
    """Block boundaries of numpy's reduction (8192) and of its pairwise leaves (128)."""
    rng = np.random.default_rng(5)
    for n in (1, 7, 8, 9, 127, 128, 129, 8191, 8192, 8193, 16384, 20000, 480000, 480001):
        pcm = rng.integers(-32768, 32768, n, dtype=np.int16)
        want = np.mean(np.square(pcm.astype(np.float32) / 32768.0))
        assert ingest.mean_square(pcm) == want, n
    st = rng.integers(-20000, 20000, 2 * 9001, dtype=np.int16)
    mono = st.astype(np.float32).reshape(-1, 2) / 32768.0
    assert ingest.mean_square(st, channels=2) == np.mean(np.square(mono.mean(axis=1)))
