"""ORACLE (test infrastructure only) — Whisper encoder / decoder in numpy.

Restates the network CTranslate2 runs for ``WhisperModel`` (upstream, not vendored;
structure as in transformers ``models/whisper/modeling_whisper.py:241-279`` (attention,
k_proj without bias), ``:566-642`` (encoder), ``:649-790`` (decoder), ``:965-970``
(tied logits projection)).  Weights use the canonical layout of
``open-speech_amd/weights.py``.

``fp16=True`` rounds activations to fp16 at exactly the points where the HIP path
stores fp16 (``GPU_POINTS``: encoder GEMM inputs, attention probabilities fed to the
MFMA, K/V caches, decoder q), with
fp32 accumulation everywhere and an fp32 residual stream, so the comparison with
the GPU isolates accumulation-order effects.  ``fp16=False`` is plain fp32/fp64 math
and is what transformers' fp32 model computes.  ``fp16`` may also be a collection of
rounding-point names (``ROUND_POINTS``): only those points round, which is how
``tools/precision_study.py`` finds the point that dominates the logits error.
"""
from __future__ import annotations

import numpy as np
from scipy.special import erf


def _h(x, on=True):
    return x.astype(np.float16).astype(np.float32) if on else x.astype(np.float32)


# every place an fp16 Whisper pipeline may store an activation in fp16
ROUND_POINTS = frozenset({
    "mel", "conv1", "enc_ln", "enc_qkv", "enc_p", "enc_attn", "enc_fc1", "enc_out",  # encoder
    "xkv",                                                                           # cross K/V
    "dec_ln", "dec_qkv", "dec_attn", "dec_q", "dec_fc1", "dec_final_ln",             # decoder
})
# the points where the HIP path DOES round: the decoder's GEMM operands
# (LayerNorm outputs, attention outputs, GELU outputs) are hi/lo fp16 pairs, i.e. fp32-
# accurate, because rounding them cost 1.5e-3 of log-softmax at turbo dims
# (tools/precision_study.py); q, the self-K/V cache and the cross-K/V stay fp16.
GPU_POINTS = ROUND_POINTS - {"dec_ln", "dec_attn", "dec_fc1", "dec_final_ln"}


def layer_norm(x, g, b, eps=1e-5):
    x64 = x.astype(np.float64)
    mu = x64.mean(-1, keepdims=True)
    var = ((x64 - mu) ** 2).mean(-1, keepdims=True)
    return ((x64 - mu) / np.sqrt(var + eps) * g + b).astype(np.float32)


def gelu(x):
    x64 = x.astype(np.float64)
    return (0.5 * x64 * (1.0 + erf(x64 / np.sqrt(2.0)))).astype(np.float32)


def attention(q, k, v, n_head, round_p, fp16):
    """q [Tq, D], k/v [Tk, D] -> [Tq, D]; softmax(q kᵀ / sqrt(64)) v per head."""
    Tq, D = q.shape
    hd = D // n_head
    out = np.empty((Tq, D), np.float32)
    scale = np.float32(hd ** -0.5)
    for h in range(n_head):
        sl = slice(h * hd, (h + 1) * hd)
        s = (q[:, sl] @ k[:, sl].T) * scale
        m = s.max(-1, keepdims=True)
        p = np.exp((s - m).astype(np.float64)).astype(np.float32)
        l = p.sum(-1, keepdims=True, dtype=np.float64).astype(np.float32)
        pv = _h(p, round_p and fp16) @ v[:, sl]
        out[:, sl] = pv / l
    return out


class WhisperOracle:
    def __init__(self, dims, weights: dict, fp16=True):
        self.d = dims
        if fp16 is True or fp16 is False:
            self.points = GPU_POINTS if fp16 else frozenset()
        else:
            self.points = frozenset(fp16)
            assert self.points <= ROUND_POINTS, self.points - ROUND_POINTS
        self.fp16 = bool(self.points)
        self.w = {k: (v.astype(np.float32) if v.dtype == np.float16 else v) for k, v in weights.items()}

    # ---------------- encoder ----------------
    def encode(self, mel_window: np.ndarray) -> np.ndarray:
        """mel_window [n_mels, 3000] (normalized) -> encoder output [1500, D] (fp16-valued fp32)."""
        d, w, r = self.d, self.w, self.points
        n_mels, T = mel_window.shape
        x1 = np.zeros((T + 2, n_mels), np.float32)
        x1[1:T + 1] = _h(mel_window.T, "mel" in r)
        col = np.concatenate([x1[0:T], x1[1:T + 1], x1[2:T + 2]], axis=1)         # [T, 3*n_mels]
        h1 = gelu(col @ w["enc.conv1.w"].reshape(d.n_audio_state, -1).T + w["enc.conv1.b"])
        h1p = np.zeros((T + 1, d.n_audio_state), np.float32)
        h1p[1:] = _h(h1, "conv1" in r)
        T2 = T // 2
        col2 = np.stack([h1p[2 * t:2 * t + 3].reshape(-1) for t in range(T2)])   # [T2, 3D]
        x = gelu(col2 @ w["enc.conv2.w"].reshape(d.n_audio_state, -1).T + w["enc.conv2.b"])
        x = x + w["enc.pos"][:T2]
        for i in range(d.n_audio_layer):
            x = self.encoder_layer(i, x)
        return _h(layer_norm(x, w["enc.lnpost.g"], w["enc.lnpost.b"]), "enc_out" in r)

    def encoder_layer(self, i: int, x: np.ndarray) -> np.ndarray:
        """One pre-LN encoder block on the fp32 residual stream x [T, D]."""
        d, w, r = self.d, self.w, self.points
        D = d.n_audio_state
        p = f"enc.l{i}"
        xn = _h(layer_norm(x, w[p + ".ln1.g"], w[p + ".ln1.b"]), "enc_ln" in r)
        qkv = _h(xn @ w[p + ".qkv.w"].T + w[p + ".qkv.b"], "enc_qkv" in r)
        o = _h(attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], d.n_audio_head, True, "enc_p" in r),
               "enc_attn" in r)
        x = x + (o @ w[p + ".o.w"].T + w[p + ".o.b"])
        xn = _h(layer_norm(x, w[p + ".ln2.g"], w[p + ".ln2.b"]), "enc_ln" in r)
        hdn = _h(gelu(xn @ w[p + ".fc1.w"].T + w[p + ".fc1.b"]), "enc_fc1" in r)
        return x + (hdn @ w[p + ".fc2.w"].T + w[p + ".fc2.b"])

    def cross_kv(self, enc: np.ndarray) -> np.ndarray:
        """[L, 2, 1500, D] cross-attention keys/values (fp16-valued)."""
        d = self.d
        kv = _h(enc @ self.w["dec.crosskv.w"].T + self.w["dec.crosskv.b"], "xkv" in self.points)
        return kv.reshape(enc.shape[0], d.n_text_layer, 2, d.n_text_state).transpose(1, 2, 0, 3).copy()

    # ---------------- decoder ----------------
    def new_cache(self):
        d = self.d
        return {"k": np.zeros((d.n_text_layer, d.n_text_ctx, d.n_text_state), np.float32),
                "v": np.zeros((d.n_text_layer, d.n_text_ctx, d.n_text_state), np.float32)}

    def decoder_step(self, token: int, pos: int, cache: dict, xkv: np.ndarray) -> np.ndarray:
        """One token through the decoder; returns fp32 logits [n_vocab]."""
        d, w, r = self.d, self.w, self.points
        D = d.n_text_state
        x = (w["dec.tok"][token] + w["dec.pos"][pos])[None, :].astype(np.float32)
        for i in range(d.n_text_layer):
            p = f"dec.l{i}"
            xn = _h(layer_norm(x, w[p + ".ln1.g"], w[p + ".ln1.b"]), "dec_ln" in r)
            qkv = _h(xn @ w[p + ".qkv.w"].T + w[p + ".qkv.b"], "dec_qkv" in r)
            cache["k"][i, pos] = qkv[0, D:2 * D]
            cache["v"][i, pos] = qkv[0, 2 * D:]
            o = _h(attention(qkv[:, :D], cache["k"][i, :pos + 1], cache["v"][i, :pos + 1],
                             d.n_text_head, False, False), "dec_attn" in r)
            x = x + (o @ w[p + ".o.w"].T + w[p + ".o.b"])
            xn = _h(layer_norm(x, w[p + ".ln2.g"], w[p + ".ln2.b"]), "dec_ln" in r)
            q = _h(xn @ w[p + ".xq.w"].T + w[p + ".xq.b"], "dec_q" in r)
            o = _h(attention(q, xkv[i, 0], xkv[i, 1], d.n_text_head, False, False), "dec_attn" in r)
            x = x + (o @ w[p + ".xo.w"].T + w[p + ".xo.b"])
            xn = _h(layer_norm(x, w[p + ".ln3.g"], w[p + ".ln3.b"]), "dec_ln" in r)
            hdn = _h(gelu(xn @ w[p + ".fc1.w"].T + w[p + ".fc1.b"]), "dec_fc1" in r)
            x = x + (hdn @ w[p + ".fc2.w"].T + w[p + ".fc2.b"])
        h = _h(layer_norm(x, w["dec.lnpost.g"], w["dec.lnpost.b"]), "dec_final_ln" in r)
        return (h @ w["dec.tok"].T)[0].astype(np.float32)
