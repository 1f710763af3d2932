"""GPU drop-ins for the reference's audio ingest, byte-identical to it.

* ``preprocess_stt_audio(wav_bytes, *, noise_reduce, normalize)`` replaces
  ``src/audio/preprocessing.py:53-63`` (called at ``src/main.py:296-300``).
* ``resample_pcm16(pcm_bytes, from_rate, to_rate)`` replaces
  ``src/streaming.py:55-91`` (called at ``src/streaming.py:293-294`` on every 100 ms
  client chunk).

The per-sample work runs in HIP (``csrc/ingest.hip`` through ``osw_ingest_*``); the
host keeps what the reference's control flow needs: the RIFF header (the ``wave``
module, so malformed / non-16-bit input takes the same exception path and is
returned unchanged), the float32 scalar chain of ``normalize_gain`` (numpy, the
same expressions on the GPU's bit-exact mean square), and scipy's filter design
(``firwin``, what ``resample_poly`` designs).  Pinned against the reference's own
outputs by tests/test_ref_fixtures_gpu.py (fixtures: tools/make_ref_fixtures.py).
"""
from __future__ import annotations

import ctypes as C
import io
import wave
from functools import lru_cache
from math import gcd

import numpy as np

from . import _lib

DEVICE = 0


def _i16p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int16))


def _read_wav(wav_bytes: bytes):
    """wav_bytes_to_float32_mono's parsing (preprocessing.py:9-20), samples left as int16."""
    with wave.open(io.BytesIO(wav_bytes), "rb") as wf:
        sr = wf.getframerate()
        channels = wf.getnchannels()
        width = wf.getsampwidth()
        raw = wf.readframes(wf.getnframes())
    if width != 2:
        raise ValueError("Only 16-bit WAV is supported for preprocessing")
    return np.frombuffer(raw, dtype=np.int16), sr, channels


def mean_square(pcm: np.ndarray, channels: int = 1, device: int = DEVICE) -> np.float32:
    """np.mean(np.square(mono)) of int16 PCM as numpy computes it (float32, its order)."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    n = pcm.size // channels
    if n == 0:
        return np.float32(np.nan)   # numpy: mean of an empty slice
    out = C.c_float()
    _lib.check(_lib.load().osw_ingest_mean_square(device, _i16p(pcm), n, channels, C.byref(out)),
               "osw_ingest_mean_square")
    return np.float32(out.value)


def gain_for(ms: np.float32, target_dbfs: float = -18.0):
    """normalize_gain's scalar chain (preprocessing.py:36-41) on float32 scalars; None = skipped."""
    rms = np.sqrt(ms)
    if rms <= 1e-8:
        return None
    current_dbfs = 20 * np.log10(rms)
    gain_db = target_dbfs - current_dbfs
    return 10 ** (gain_db / 20)


def normalize_pcm16(pcm: np.ndarray, channels: int = 1, normalize: bool = True, device: int = DEVICE) -> np.ndarray:
    """int16 PCM -> the int16 samples preprocess_stt_audio writes back."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    n = pcm.size // channels
    if n == 0:
        return np.zeros(0, np.int16)
    g = gain_for(mean_square(pcm, channels, device)) if normalize else None
    out = np.empty(n, np.int16)
    _lib.check(_lib.load().osw_ingest_apply_gain(device, _i16p(pcm), n, channels, 0 if g is None else 1,
                                                 0.0 if g is None else float(g), _i16p(out)), "osw_ingest_apply_gain")
    return out


def _write_wav(pcm: np.ndarray, sr: int) -> bytes:
    buf = io.BytesIO()
    with wave.open(buf, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sr)
        wf.writeframes(pcm.tobytes())
    return buf.getvalue()


def preprocess_stt_audio(wav_bytes: bytes, *, noise_reduce: bool, normalize: bool, device: int = DEVICE) -> bytes:
    try:
        pcm, sr, channels = _read_wav(wav_bytes)
    except Exception:
        # the reference returns non-WAV / non-16-bit input unchanged (preprocessing.py:54-58)
        return wav_bytes
    if noise_reduce:
        return _write_wav(_denoised_pcm16(pcm, sr, channels, normalize), sr)
    return _write_wav(normalize_pcm16(pcm, channels, normalize, device), sr)


def _denoised_pcm16(pcm: np.ndarray, sr: int, channels: int, normalize: bool) -> np.ndarray:
    """STT_NOISE_REDUCE (src/config.py:166): the reference's chain on the host,
    preprocessing.py:59-63 — float32 mono, noisereduce's spectral gating (a host
    library, as in the reference), normalize_gain, clip, x 32767, truncating cast.
    The gain is applied to the denoised float signal, so it stays in numpy here (the
    GPU gain kernel takes int16 input); the same RuntimeError as the reference when the
    optional dependency is absent."""
    try:
        import noisereduce as nr  # type: ignore
    except ImportError as e:
        raise RuntimeError("Noise reduction requires optional dependency: pip install 'open-speech[noise]'") from e
    audio = pcm.astype(np.float32) / 32768.0
    if channels > 1:
        audio = audio.reshape(-1, channels).mean(axis=1)
    audio = nr.reduce_noise(y=audio, sr=sr)
    if normalize:
        rms = np.sqrt(np.mean(np.square(audio)))
        if rms > 1e-8:
            gain = 10 ** ((-18.0 - 20 * np.log10(rms)) / 20)
            audio = np.clip(audio * gain, -1.0, 1.0)
    return (np.clip(audio, -1.0, 1.0) * 32767.0).astype(np.int16)


@lru_cache(maxsize=32)
def _filter(up: int, down: int) -> np.ndarray:
    """resample_poly's default FIR: firwin(2*half_len+1, 1/max_rate, kaiser 5.0) as float32, times up."""
    from scipy.signal import firwin
    max_rate = max(up, down)
    h = firwin(2 * 10 * max_rate + 1, 1.0 / max_rate, window=("kaiser", 5.0)).astype(np.float32)
    h *= up
    h.setflags(write=False)
    return h


def resample_int16(x: np.ndarray, up: int, down: int, device: int = DEVICE) -> np.ndarray:
    """resample_poly(x.astype(float32), up, down, padtype="line") clipped and truncated to int16."""
    g = gcd(up, down)
    up, down = up // g, down // g
    x = np.ascontiguousarray(x, dtype=np.int16)
    n_out = -(-x.size * up // down)
    h = _filter(up, down)
    out = np.empty(n_out, np.int16)
    _lib.check(_lib.load().osw_ingest_resample(device, _i16p(x), x.size, up, down,
                                               h.ctypes.data_as(C.POINTER(C.c_float)), h.size, _i16p(out), n_out),
               "osw_ingest_resample")
    return out


def resample_pcm16(pcm_bytes: bytes, from_rate: int, to_rate: int, device: int = DEVICE) -> bytes:
    if from_rate == to_rate:
        return pcm_bytes
    samples = np.frombuffer(pcm_bytes, dtype=np.int16)
    if len(samples) == 0:
        return pcm_bytes
    if len(samples) == 1:
        out_len = int(len(samples) * (to_rate / from_rate))
        if out_len <= 0:
            return b""
        return np.full(out_len, samples[0], dtype=np.int16).tobytes()
    g = gcd(to_rate, from_rate)
    return resample_int16(samples, to_rate // g, from_rate // g, device).tobytes()
