"""Deterministic inputs for the reference-pinned fixtures (tools/make_ref_fixtures.py
writes the reference's outputs for them; tests/test_ref_fixtures_*.py regenerate the
same inputs and compare).  Covers the shapes the reference's ingest sees: 16 kHz
mono WAVs from ffmpeg (``src/utils/audio.py:22-34``), quiet / clipping / silent
clips, stereo, other rates, malformed and non-16-bit WAVs, and the streaming path's
100 ms client-rate chunks (``src/streaming.py:285-294``)."""
from __future__ import annotations

import io
import wave

import numpy as np

from open_speech_amd.synth import chirp_clip, to_wav_bytes


def _wav(pcm: np.ndarray, sr: int, ch: int = 1, width: int = 2) -> bytes:
    buf = io.BytesIO()
    with wave.open(buf, "wb") as wf:
        wf.setnchannels(ch)
        wf.setsampwidth(width)
        wf.setframerate(sr)
        wf.writeframes(np.ascontiguousarray(pcm).tobytes())
    return buf.getvalue()


def _scaled(i: int, seconds: float, gain: float) -> np.ndarray:
    x = chirp_clip(i, seconds).astype(np.float64) * gain
    return np.clip(np.round(x), -32768, 32767).astype(np.int16)


def _tone(sr: int, seconds: float, freq: float, amp: float, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.arange(int(round(seconds * sr))) / sr
    x = amp * np.sin(2 * np.pi * freq * t + rng.uniform(0, 6.28)) + rng.standard_normal(t.size) * amp * 0.05
    return np.clip(np.round(x * 32767), -32768, 32767).astype(np.int16)


def preprocess_cases():
    """(name, wav bytes) for preprocess_stt_audio."""
    yield "chirp30", to_wav_bytes(chirp_clip(0, 30.0))
    yield "quiet7", to_wav_bytes(_scaled(1, 7.3, 0.1))
    yield "loud3", to_wav_bytes(_scaled(2, 3.0, 12.0))            # gain < 1 after clipping-level input
    yield "silence2", to_wav_bytes(np.zeros(32000, np.int16))      # rms <= 1e-8: gain skipped
    yield "tiny1", to_wav_bytes(np.array([1234], np.int16))
    yield "dc05", to_wav_bytes(np.full(8000, -700, np.int16))
    st = np.stack([_scaled(3, 2.0, 0.5), _scaled(4, 2.0, 0.3)], axis=1)
    yield "stereo2", _wav(st, 16000, ch=2)
    yield "rate44k", _wav(_tone(44100, 1.5, 300.0, 0.2, 5), 44100)
    yield "u8", _wav(np.full(1600, 128, np.uint8), 16000, width=1)   # ValueError -> input returned
    yield "notwav", b"RIFF" + b"\x00" * 100                          # the reference tests' upload
    yield "empty_data", to_wav_bytes(np.zeros(0, np.int16))


def noise_cases():
    """(name, wav bytes) for preprocess_stt_audio(noise_reduce=True)."""
    yield "chirp30", to_wav_bytes(chirp_clip(0, 30.0))
    st = np.stack([_scaled(3, 2.0, 0.5), _scaled(4, 2.0, 0.3)], axis=1)
    yield "stereo2", _wav(st, 16000, ch=2)
    yield "silence2", to_wav_bytes(np.zeros(32000, np.int16))


def standin_reduce_noise(y: np.ndarray, sr: int) -> np.ndarray:
    """A deterministic stand-in for ``noisereduce.reduce_noise`` (the optional
    dependency is absent on both machines): halves the signal and adds a fixed
    low-level tone, so the chain around it (float32 mono in, gain + clip + truncating
    cast out) is what the fixture pins."""
    t = np.arange(y.size, dtype=np.float32)
    return (y * np.float32(0.5) + np.float32(0.01) * np.sin(t * np.float32(0.01))).astype(np.float32)


def resample_cases():
    """(name, pcm16 bytes, from_rate, to_rate) for resample_pcm16."""
    for sr, secs in ((8000, 2.0), (22050, 1.5), (44100, 2.0), (48000, 3.0), (11025, 0.7), (32000, 1.0)):
        yield f"r{sr}_{secs}", _tone(sr, secs, 440.0, 0.4, sr).tobytes(), sr, 16000
    # the streaming path resamples each 100 ms client chunk on its own (src/streaming.py:285-294)
    for sr in (48000, 44100, 8000, 96000):
        n = sr // 10
        yield f"chunk{sr}", _tone(sr, n / sr, 1000.0, 0.9, 7 + sr).tobytes(), sr, 16000
    yield "loud48k", _tone(48000, 0.5, 200.0, 1.0, 3).tobytes(), 48000, 16000   # overshoot -> clip
    yield "one48k", np.array([999], np.int16).tobytes(), 48000, 16000
    yield "one8k", np.array([-5], np.int16).tobytes(), 8000, 16000
    yield "two8k", np.array([100, -100], np.int16).tobytes(), 8000, 16000
    yield "empty", b"", 44100, 16000
    yield "same", _tone(16000, 0.25, 500.0, 0.5, 1).tobytes(), 16000, 16000


def subtitle_segments():
    """(start, end, text) tuples: rounding edges of the srt / vtt time formatters."""
    return [(0.0, 2.5, " Hello there."), (2.5, 61.004, "world  "), (0.1 + 0.2, 7.0000001, "a"),
            (59.999, 60.0, " edge"), (3599.9995, 3661.5, " past an hour "), (7322.123, 7323.987, "x"),
            (1.005, 1.015, " ms"), (10.07, 12.34, ""), (0.02 * 1499, 30.0, " last")]
