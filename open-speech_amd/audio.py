"""Audio ingest for the backend: the bytes ``transcribe()`` receives -> int16 mono 16 kHz.

The reference hands faster-whisper a temp WAV file (``src/backends/faster_whisper.py:231-245``)
which it decodes with PyAV to float32 mono 16 kHz (``decode_audio``: s16 samples / 32768).
The REST endpoint already converted the upload with ffmpeg to 16 kHz mono s16 WAV
(``src/utils/audio.py:10-38``) and gain-normalised it (``src/audio/preprocessing.py:53-63``),
so the common case is a plain PCM16 WAV that is parsed here in memory (no temp file).
Other sample rates / channel counts are mixed down (channel mean) and resampled
(polyphase); other containers go through ffmpeg like ``convert_to_wav``.
"""
from __future__ import annotations

import io
import shutil
import struct
import subprocess
import wave
from math import gcd

import numpy as np

SR = 16000


def _resample(x: np.ndarray, sr: int) -> np.ndarray:
    if sr == SR:
        return x
    from scipy.signal import resample_poly

    g = gcd(sr, SR)
    return resample_poly(x, SR // g, sr // g)


def pcm16_from_wav(data: bytes) -> np.ndarray:
    """Parse a RIFF/WAVE PCM buffer to int16 mono 16 kHz."""
    with wave.open(io.BytesIO(data), "rb") as wf:
        sr, ch, width = wf.getframerate(), wf.getnchannels(), wf.getsampwidth()
        raw = wf.readframes(wf.getnframes())
    if width == 2:
        x = np.frombuffer(raw, dtype="<i2")
    elif width == 4:
        x = (np.frombuffer(raw, dtype="<i4") >> 16).astype(np.int16)
    elif width == 1:
        x = ((np.frombuffer(raw, dtype=np.uint8).astype(np.int16) - 128) << 8).astype(np.int16)
    else:
        raise ValueError(f"unsupported WAV sample width {width}")
    if ch > 1:
        x = x.reshape(-1, ch).astype(np.float32).mean(axis=1)
        if sr == SR:
            return np.clip(np.round(x), -32768, 32767).astype(np.int16)
    if sr == SR:
        return np.ascontiguousarray(x, dtype=np.int16)
    y = _resample(x.astype(np.float32), sr)
    return np.clip(np.round(y), -32768, 32767).astype(np.int16)


def decode_audio_bytes(data: bytes) -> np.ndarray:
    """Bytes of any container -> int16 mono 16 kHz (WAV in memory, else ffmpeg)."""
    if len(data) >= 12 and data[:4] == b"RIFF" and data[8:12] == b"WAVE":
        try:
            return pcm16_from_wav(data)
        except (wave.Error, EOFError) as e:
            raise ValueError(f"invalid WAV data: {e}") from e
    if shutil.which("ffmpeg") is None:
        raise ValueError("audio is not a PCM WAV and ffmpeg is not available to convert it")
    p = subprocess.run(["ffmpeg", "-nostdin", "-i", "pipe:0", "-f", "s16le", "-ac", "1", "-ar", str(SR), "pipe:1"],
                       input=data, capture_output=True, check=False)
    if p.returncode != 0:
        raise ValueError("ffmpeg could not decode the audio: " + p.stderr.decode(errors="replace")[-300:])
    return np.frombuffer(p.stdout, dtype="<i2").copy()


def pcm_to_wav(pcm: bytes, sample_rate: int) -> bytes:
    """RIFF header + PCM16 mono, byte-identical to ``StreamingSession._pcm_to_wav``
    (``src/streaming.py:494-516``; pinned by tests/test_ref_fixtures_cpu.py)."""
    n = len(pcm)
    return struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + n, b"WAVE", b"fmt ", 16, 1, 1, sample_rate,
                       sample_rate * 2, 2, 16, b"data", n) + pcm
