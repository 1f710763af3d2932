"""Synthetic 16 kHz mono int16 clips (BASELINE.md §3 / SURVEY.md §8d).

Each clip: a sum of 3 log-swept chirps (100 Hz → 4 kHz, random phases) plus white
noise at −30 dB, amplitude-modulated at a 4 Hz syllable rate, RMS-normalised to
−18 dBFS (the target of ``src/audio/preprocessing.py:35``).  Seeded by
``numpy.random.default_rng(1234 + i)``.
"""
from __future__ import annotations

import io
import wave

import numpy as np

SR = 16000


def chirp_clip(i: int, seconds: float = 30.0) -> np.ndarray:
    rng = np.random.default_rng(1234 + i)
    n = int(round(seconds * SR))
    t = np.arange(n, dtype=np.float64) / SR
    f0, f1 = 100.0, 4000.0
    T = max(seconds, 1e-3)
    k = np.log(f1 / f0)
    sig = np.zeros(n)
    for _ in range(3):
        ph = rng.uniform(0, 2 * np.pi)
        # duration of one sweep is random in [2, 8] s, repeated
        dur = rng.uniform(2.0, 8.0)
        tt = np.mod(t + rng.uniform(0, dur), dur)
        phase = 2 * np.pi * f0 * dur / k * (np.exp(k * tt / dur) - 1.0)
        sig += np.sin(phase + ph)
    sig /= 3.0
    sig += rng.standard_normal(n) * (10 ** (-30 / 20)) * np.sqrt(np.mean(sig ** 2) + 1e-12)
    am = 0.55 + 0.45 * np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 2 * np.pi))
    sig *= am
    del T
    return _to_int16_at_dbfs(sig, -18.0)


def tone_clip(seconds: float = 7.3, freq: float = 440.0) -> np.ndarray:
    t = np.arange(int(round(seconds * SR))) / SR
    return _to_int16_at_dbfs(np.sin(2 * np.pi * freq * t), -18.0)


def noise_clip(i: int, seconds: float = 30.0) -> np.ndarray:
    """White noise at -18 dBFS, seeded by ``numpy.random.default_rng(i)``."""
    x = np.random.default_rng(i).standard_normal(int(round(seconds * SR)))
    return _to_int16_at_dbfs(x, -18.0)


def silence_clip(seconds: float = 5.0) -> np.ndarray:
    return np.zeros(int(round(seconds * SR)), dtype=np.int16)


def _to_int16_at_dbfs(x: np.ndarray, dbfs: float) -> np.ndarray:
    rms = np.sqrt(np.mean(x ** 2))
    if rms > 0:
        x = x * (10 ** (dbfs / 20) / rms)
    return (np.clip(x, -1.0, 1.0) * 32767.0).astype(np.int16)


def to_wav_bytes(pcm: np.ndarray, sr: int = SR) -> bytes:
    buf = io.BytesIO()
    with wave.open(buf, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sr)
        wf.writeframes(np.asarray(pcm, dtype=np.int16).tobytes())
    return buf.getvalue()
