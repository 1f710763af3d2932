"""ORACLE (test infrastructure only) — the reference's audio ingest, restated step by
step in float32 so that each rounding is explicit (the HIP ingest kernels must
reproduce these bits):

* ``preprocess_stt_audio`` — /root/reference/src/audio/preprocessing.py:53-63:
  int16 / 32768 (``wav_bytes_to_float32_mono`` :9-20, channel mean for stereo),
  ``normalize_gain`` :35-42 (rms = sqrt(mean(square(audio))) with numpy's float32
  pairwise summation, dBFS, gain to -18 dBFS, clip to ±1),
  ``float32_mono_to_wav_bytes`` :23-32 (clip, ×32767, truncating astype(int16)).
  numpy 2.x sums a contiguous float32 array in blocks of 8192 elements (the ufunc
  buffer), each block by ``pairwise_sum`` (numpy/_core/src/umath/loops_utils.h.src:
  leaves of <= 128 elements with 8 running sums, halving splits rounded down to a
  multiple of 8), and adds the block sums in order.
* ``resample_pcm16`` — /root/reference/src/streaming.py:55-91: scipy 1.15
  ``resample_poly(samples_f32, up, down, padtype="line")``: Kaiser(5.0) firwin of
  2·10·max(up,down)+1 taps cast to float32 and scaled by ``up``, zero pre/post pad,
  then ``upfirdn`` in mode "line" (the signal extended by the line through its first
  and last samples) — per output, a float32 multiply-then-add over the polyphase
  taps in ascending order starting from 0 — then clip to int16 range and truncate.

Pinned by tests/test_ref_fixtures_cpu.py against the reference's own outputs
(tools/make_ref_fixtures.py -> tests/golden/ref_fixtures.*).
"""
from __future__ import annotations

import io
import wave
from math import gcd

import numpy as np

F = np.float32
BLOCK = 8192      # numpy ufunc buffer size: reductions see at most this many elements per inner loop
PW_BLOCKSIZE = 128


def pairwise_sum(a: np.ndarray) -> np.float32:
    """numpy's ``FLOAT_pairwise_sum`` for one inner-loop block (float32 accumulators)."""
    n = len(a)
    if n < 8:
        r = F(0.0)
        for x in a:
            r = F(r + x)
        return r
    if n <= PW_BLOCKSIZE:
        m = n - n % 8
        r = a[:8].astype(F).copy()
        for i in range(8, m, 8):
            r = (r + a[i:i + 8]).astype(F)
        res = F(F(F(r[0] + r[1]) + F(r[2] + r[3])) + F(F(r[4] + r[5]) + F(r[6] + r[7])))
        for i in range(m, n):
            res = F(res + a[i])
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return F(pairwise_sum(a[:n2]) + pairwise_sum(a[n2:]))


def float32_sum(a: np.ndarray) -> np.float32:
    """np.add.reduce of a contiguous float32 vector: per-8192 block pairwise sums, added in order."""
    a = np.ascontiguousarray(a, dtype=F)
    if a.size == 0:
        return F(0.0)
    acc = None
    for lo in range(0, a.size, BLOCK):
        s = pairwise_sum(a[lo:lo + BLOCK])
        acc = s if acc is None else F(acc + s)
    return acc


def float32_mean(a: np.ndarray) -> np.float32:
    return F(float32_sum(a) / F(a.size)) if a.size else F(np.nan)


def wav_to_float32_mono(wav: bytes):
    with wave.open(io.BytesIO(wav), "rb") as wf:
        sr, ch, width = wf.getframerate(), wf.getnchannels(), wf.getsampwidth()
        raw = wf.readframes(wf.getnframes())
    if width != 2:
        raise ValueError("Only 16-bit WAV is supported for preprocessing")
    x = np.frombuffer(raw, dtype=np.int16).astype(F) / F(32768.0)
    if ch > 1:   # mean over the channel axis: sequential float32 adds, then / ch
        x = x.reshape(-1, ch)
        s = x[:, 0].copy()
        for c in range(1, ch):
            s = (s + x[:, c]).astype(F)
        x = (s / F(ch)).astype(F)
    return x, sr


def gain_for(audio: np.ndarray, target_dbfs: float = -18.0):
    """The scalar chain of normalize_gain: None when the gain step is skipped."""
    rms = np.sqrt(float32_mean(np.square(audio)))
    if rms <= 1e-8:
        return None
    current_dbfs = 20 * np.log10(rms)
    gain_db = target_dbfs - current_dbfs
    return 10 ** (gain_db / 20)


def preprocess_stt_audio(wav: bytes, *, noise_reduce: bool = False, normalize: bool = True) -> bytes:
    if noise_reduce:
        raise NotImplementedError("noise reduction is an optional dependency of the reference")
    try:
        audio, sr = wav_to_float32_mono(wav)
    except Exception:
        return wav
    if normalize:
        g = gain_for(audio)
        if g is not None:
            audio = np.clip((audio * g).astype(F), F(-1.0), F(1.0))
    pcm = (np.clip(audio, F(-1.0), F(1.0)) * F(32767.0)).astype(np.int16)
    buf = io.BytesIO()
    with wave.open(buf, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sr)
        wf.writeframes(pcm.tobytes())
    return buf.getvalue()


# ---------------------------------------------------------------- resampling
def poly_filter(up: int, down: int) -> np.ndarray:
    """resample_poly's default filter: firwin(2*half_len+1, 1/max, kaiser 5.0) -> float32 * up."""
    from scipy.signal import firwin
    max_rate = max(up, down)
    half_len = 10 * max_rate
    h = firwin(2 * half_len + 1, 1.0 / max_rate, window=("kaiser", 5.0)).astype(F)
    h *= up
    return h


def upfirdn_output_len(len_h: int, n_in: int, up: int, down: int) -> int:
    n = (n_in + (len_h + (-len_h % up)) // up - 1) * up
    return n // down + (1 if n % down else 0)


def resample_poly_line(x: np.ndarray, up: int, down: int) -> np.ndarray:
    """scipy.signal.resample_poly(x_f32, up, down, padtype='line') restated (float32)."""
    g = gcd(up, down)
    up //= g
    down //= g
    x = np.ascontiguousarray(x, dtype=F)
    n_in = x.size
    n_out = n_in * up
    n_out = n_out // down + (1 if n_out % down else 0)
    h = poly_filter(up, down)
    half_len = (len(h) - 1) // 2
    n_pre_pad = down - half_len % down
    n_post_pad = 0
    n_pre_remove = (half_len + n_pre_pad) // down
    while upfirdn_output_len(len(h) + n_pre_pad + n_post_pad, n_in, up, down) < n_out + n_pre_remove:
        n_post_pad += 1
    hp = np.concatenate([np.zeros(n_pre_pad, F), h, np.zeros(n_post_pad, F)])
    len_h = hp.size
    pad = len_h + (-len_h % up)
    htf = np.zeros(pad, F)
    htf[:len_h] = hp
    htf = htf.reshape(-1, up).T[:, ::-1].ravel()       # _pad_h: transposed, flipped phases
    hpp = pad // up
    # upfirdn "line" extension: the line through x[0] and x[-1]
    slope = F((x[-1] - x[0]) / F(n_in - 1))

    def xval(i: np.ndarray) -> np.ndarray:
        v = x[np.clip(i, 0, n_in - 1)].copy()
        lo, hi = i < 0, i >= n_in
        v[lo] = (x[0] + (i[lo].astype(F) * slope).astype(F)).astype(F)
        v[hi] = (x[-1] + ((i[hi] - n_in + 1).astype(F) * slope).astype(F)).astype(F)
        return v

    # the (x_idx, phase) walk of upfirdn for the kept outputs
    ys = np.arange(n_pre_remove, n_pre_remove + n_out, dtype=np.int64)
    tt = ys * down                      # t before the modulo, accumulated
    x_idx = tt // up
    t = tt % up
    acc = np.zeros(n_out, F)
    for j in range(hpp):
        xi = x_idx - hpp + 1 + j
        acc = (acc + (xval(xi) * htf[t * hpp + j]).astype(F)).astype(F)
    return acc


def resample_pcm16(pcm: bytes, from_rate: int, to_rate: int) -> bytes:
    if from_rate == to_rate:
        return pcm
    s = np.frombuffer(pcm, dtype=np.int16).astype(F)
    if s.size == 0:
        return pcm
    if s.size == 1:
        n = int(1 * (to_rate / from_rate))
        return b"" if n <= 0 else np.full(n, s[0], dtype=np.int16).tobytes()
    g = gcd(to_rate, from_rate)
    y = resample_poly_line(s, to_rate // g, from_rate // g)
    return np.clip(y, -32768, 32767).astype(np.int16).tobytes()
