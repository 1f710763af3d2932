"""ORACLE (test infrastructure only) — log-mel front end.

Restates faster-whisper 1.2.1 ``faster_whisper/feature_extractor.py``
(``FeatureExtractor.__call__`` / ``get_mel_filters`` / ``stft``; upstream, not
vendored — SURVEY.md §8a row a8) in float64 numpy:

  x  = pcm_int16 / 32768                       (faster_whisper.audio.decode_audio)
  x  = pad(x, (0, 160))                        (``padding=160``)
  S  = |rfft(hann_periodic(400) · frame_t)|²   centre reflect-pad 200, hop 160
  S  = S[:, :-1]                               (last frame dropped)
  M  = F_slaney[n_mels × 201] · S
  L  = log10(max(M, 1e-10));  L = max(L, max(L) − 8);  L = (L + 4) / 4

The max is taken over the whole file (all frames), as faster-whisper computes
features once per file before the 30 s seek loop.  Pinned against transformers'
``WhisperFeatureExtractor._np_extract_fbank_features`` on the same 160-padded
waveform (tools/make_golden.py → tests/golden/mel_*.npz).
"""
from __future__ import annotations

import numpy as np

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160


def hz_to_mel_slaney(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, mels)


def mel_to_hz_slaney(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filters(n_mels: int, sr: int = SAMPLE_RATE, n_fft: int = N_FFT) -> np.ndarray:
    """librosa-style slaney mel bank [n_mels, 1 + n_fft//2] (faster-whisper get_mel_filters)."""
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = mel_to_hz_slaney(np.linspace(hz_to_mel_slaney(0.0), hz_to_mel_slaney(sr / 2.0), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    return w * enorm[:, None]


def hann_periodic(n: int = N_FFT) -> np.ndarray:
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def pcm16_to_float(pcm: np.ndarray) -> np.ndarray:
    return np.asarray(pcm, dtype=np.int16).astype(np.float32) / np.float32(32768.0)


def n_frames_for(n_samples: int, padding: int = 160) -> int:
    """Frames kept by faster-whisper for n samples: 1 + (n+padding)//hop, minus the last."""
    return (n_samples + padding) // HOP


def power_spectrum(x: np.ndarray) -> np.ndarray:
    """Centred (reflect) STFT power, [201, 1 + len(x)//160], float64."""
    x = np.asarray(x, dtype=np.float64)
    xp = np.pad(x, (N_FFT // 2, N_FFT // 2), mode="reflect")
    n_frames = 1 + len(x) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(n_frames)[:, None]
    frames = xp[idx] * hann_periodic()[None, :]
    spec = np.fft.rfft(frames, axis=1)
    return (spec.real ** 2 + spec.imag ** 2).T


def log_mel_raw(audio: np.ndarray, n_mels: int, padding: int = 160) -> np.ndarray:
    """log10 mel before the per-file max clamp, [n_mels, n_frames] float64."""
    x = np.asarray(audio, dtype=np.float32)
    if padding:
        x = np.pad(x, (0, padding))
    p = power_spectrum(x)[:, :-1]
    mel = mel_filters(n_mels) @ p
    return np.log10(np.maximum(mel, 1e-10))


def log_mel(audio: np.ndarray, n_mels: int, padding: int = 160) -> np.ndarray:
    """faster-whisper FeatureExtractor.__call__ (float64): [n_mels, (n+160)//160]."""
    lg = log_mel_raw(audio, n_mels, padding)
    lg = np.maximum(lg, lg.max() - 8.0)
    return (lg + 4.0) / 4.0


def window(mel: np.ndarray, seek: int, segment_size: int, n_frames: int = 3000) -> np.ndarray:
    """``pad_or_trim(features[:, seek:seek+segment_size], 3000)`` (zero padded)."""
    seg = mel[:, seek:seek + segment_size]
    out = np.zeros((mel.shape[0], n_frames), dtype=mel.dtype)
    out[:, :seg.shape[1]] = seg[:, :n_frames]
    return out
