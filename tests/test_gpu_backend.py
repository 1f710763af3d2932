"""End-to-end through the drop-in backend on the GPU (real engine, random weights)."""
import threading

import numpy as np
import pytest

from open_speech_amd import synth
from open_speech_amd.backend import HipWhisperBackend

pytestmark = pytest.mark.gpu
MID = "random:tiny-test:1234"


@pytest.fixture(scope="module")
def backend():
    import os
    os.environ["STT_HIP_MAX_BATCH"] = "4"
    b = HipWhisperBackend()
    b.load_model(MID)
    yield b
    b.unload_model(MID)


def test_verbose_json_end_to_end(backend):
    r = backend.transcribe(synth.to_wav_bytes(synth.chirp_clip(2, 30.0)), MID, response_format="verbose_json")
    assert r["task"] == "transcribe" and abs(r["duration"] - 30.0) < 1e-6
    assert isinstance(r["language"], str) and len(r["language"]) >= 2
    for s in r["segments"]:
        # timestamps are window-relative offsets (not clamped to the duration, as upstream)
        assert 0.0 <= s["start"] <= s["end"]
        assert all(0 <= t < 51866 for t in s["tokens"])
        assert s["temperature"] == 0.0 and 0.0 <= s["no_speech_prob"] <= 1.0


def test_concurrent_equals_sequential(backend):
    wavs = [synth.to_wav_bytes(synth.chirp_clip(30 + i, 7.0 + 5 * i)) for i in range(5)]
    seq = [backend.transcribe(w, MID, response_format="verbose_json") for w in wavs]
    par = [None] * len(wavs)

    def go(i):
        par[i] = backend.transcribe(wavs[i], MID, response_format="verbose_json")
    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(wavs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for a, b in zip(seq, par):
        assert [s["tokens"] for s in a["segments"]] == [s["tokens"] for s in b["segments"]]
        assert a["language"] == b["language"]


def test_silence_and_short_clips(backend):
    for pcm in (synth.silence_clip(2.0), synth.tone_clip(0.2), np.zeros(1600, np.int16)):
        r = backend.transcribe(synth.to_wav_bytes(pcm), MID, response_format="verbose_json")
        assert "segments" in r
