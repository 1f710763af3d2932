"""Reference-pinned fixtures (tools/make_ref_fixtures.py ran the reference's OWN
functions from /root/reference): the oracle restatements and the backend's host-side
helpers must reproduce them byte for byte.

* preprocess_stt_audio  /root/reference/src/audio/preprocessing.py:53-63
* resample_pcm16        /root/reference/src/streaming.py:55-91
* _pcm_to_wav           /root/reference/src/streaming.py:494-516
* _to_srt / _to_vtt     /root/reference/src/backends/faster_whisper.py:312-344
"""
import hashlib
import json
import os
from types import SimpleNamespace

import numpy as np
import pytest

import ref_inputs
from open_speech_amd import segments
from oracle import ingest as oi

GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLD, "ref_fixtures.json")))


def sha(b):
    return hashlib.sha256(b).hexdigest()


PP = {r["name"]: r for r in META["preprocess"]}
RS = {r["name"]: r for r in META["resample"]}


@pytest.mark.parametrize("name,wav", list(ref_inputs.preprocess_cases()), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_preprocess_matches_reference(name, wav):
    rec = PP[name]
    assert sha(wav) == rec["in_sha256"], "input generator changed"
    out = oi.preprocess_stt_audio(wav, noise_reduce=False, normalize=True)
    assert len(out) == rec["out_len"]
    assert sha(out) == rec["out_sha256"], name


@pytest.mark.parametrize("case", list(ref_inputs.resample_cases()), ids=lambda c: c[0])
def test_oracle_resample_matches_reference(case):
    name, pcm, fr, to = case
    rec = RS[name]
    assert sha(pcm) == rec["in_sha256"], "input generator changed"
    out = oi.resample_pcm16(pcm, fr, to)
    assert len(out) == rec["out_len"] and sha(out) == rec["out_sha256"], name


def test_float32_sum_is_numpy_reduction():
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 127, 128, 129, 8191, 8192, 8193, 20000, 480000):
        a = rng.standard_normal(n).astype(np.float32) ** 2
        assert oi.float32_sum(a) == np.add.reduce(a), n


def test_subtitles_match_reference():
    segs = [SimpleNamespace(start=s, end=e, text=t) for s, e, t in ref_inputs.subtitle_segments()]
    assert segments.to_srt(segs) == META["srt"]
    assert segments.to_vtt(segs) == META["vtt"]
    assert segments.to_srt([]) == META["srt_empty"]
    assert segments.to_vtt([]) == META["vtt_empty"]


def test_pcm_to_wav_header_matches_reference():
    from open_speech_amd import audio
    for rec in META["pcm_to_wav"]:
        pcm = b"\x01\x02" * (rec["n_bytes"] // 2)
        h = audio.pcm_to_wav(pcm, rec["rate"])
        assert h[:44].hex() == rec["header_hex"] and sha(h) == rec["sha256"]


NOISE = {r["name"]: r for r in META["preprocess_noise"]}


@pytest.mark.parametrize("name,wav", list(ref_inputs.noise_cases()), ids=lambda v: v if isinstance(v, str) else "")
def test_noise_reduce_path_matches_reference(name, wav, monkeypatch):
    """STT_NOISE_REDUCE=true (src/config.py:166): the drop-in's preprocess_stt_audio runs
    noisereduce on the host and the reference's float chain after it; with the same
    stand-in denoiser the bytes equal the reference's own output."""
    import sys
    import types

    from open_speech_amd import ingest
    nr = types.ModuleType("noisereduce")
    nr.reduce_noise = lambda y, sr: ref_inputs.standin_reduce_noise(y, sr)
    monkeypatch.setitem(sys.modules, "noisereduce", nr)
    rec = NOISE[name]
    assert sha(wav) == rec["in_sha256"], "input generator changed"
    out = ingest.preprocess_stt_audio(wav, noise_reduce=True, normalize=True)
    assert len(out) == rec["out_len"] and sha(out) == rec["out_sha256"], name


def test_noise_reduce_without_dependency_raises_like_reference(monkeypatch):
    import sys

    from open_speech_amd import ingest
    monkeypatch.setitem(sys.modules, "noisereduce", None)    # import fails, as on both machines
    wav = next(iter(ref_inputs.noise_cases()))[1]
    with pytest.raises(RuntimeError, match=r"pip install 'open-speech\[noise\]'"):
        ingest.preprocess_stt_audio(wav, noise_reduce=True, normalize=True)
