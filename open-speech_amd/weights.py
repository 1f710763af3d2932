"""Canonical weight layout of the HIP Whisper backend, deterministic random init,
and conversion from the HuggingFace / transformers Whisper state-dict names.

The reference loads weights inside CTranslate2 (``src/backends/faster_whisper.py:40-45``);
here the host side owns the layout it uploads to the device:

* every matrix is fp16, row-major ``[out, in]`` (so every GEMM is ``A · Wᵀ``);
* conv kernels are stored tap-major ``[out, 3, in]`` so the conv stem is a GEMM
  over a contiguous 3-row window of the time-major activation;
* the encoder q/k/v projections are fused ``[3D, D]`` (k bias is zero, as Whisper's
  k_proj has no bias); the decoder cross-attention k/v of ALL layers are fused into
  one ``[L·2·D, D]`` matrix computed once per window;
* biases, LayerNorm parameters and positional tables are fp32.

Random init is a counter-based hash (splitmix64) so the same tensors can be
generated on the device (``osw_init_uniform``) and in numpy, bit for bit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .dims import WhisperDims

F16 = "f16"
F32 = "f32"


@dataclass(frozen=True)
class TensorSpec:
    name: str
    shape: tuple
    dtype: str            # "f16" | "f32"
    kind: str             # "uniform" | "sinusoid"
    scale: float = 0.0
    offset: float = 0.0
    zero_lo: int = 0      # [zero_lo, zero_hi) flat range forced to 0 (k bias)
    zero_hi: int = 0

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


def canonical_specs(d: WhisperDims, *, w_std: float = 0.02, emb_std: float = 0.02,
                    pos_std: float = 0.02, out_gain: float = 1.0) -> list[TensorSpec]:
    """All tensors of the model, in a fixed order (the index is the hash stream id).
    ``pos_std`` / ``out_gain``: the decoder's positional-embedding scale and the final
    LayerNorm's gain (the goldens raise both so that greedy decoding of random weights
    emits varied text with clear top-2 margins; tools/make_golden.py)."""
    De, Dd, M = d.n_audio_state, d.n_text_state, d.n_mels
    u = math.sqrt(3.0)  # uniform[-a, a) has std a/sqrt(3)
    W = w_std * u
    B = 0.02 * u
    G = 0.05 * u
    s: list[TensorSpec] = []

    def mat(name, shape, scale=W):
        s.append(TensorSpec(name, tuple(shape), F16, "uniform", scale))

    def vec(name, n, scale=B, offset=0.0, zero=(0, 0)):
        s.append(TensorSpec(name, (n,), F32, "uniform", scale, offset, zero[0], zero[1]))

    def ln(prefix, n):
        vec(prefix + ".g", n, G, 1.0)
        vec(prefix + ".b", n, B)

    mat("enc.conv1.w", (De, 3, M), W * 2)
    vec("enc.conv1.b", De)
    mat("enc.conv2.w", (De, 3, De))
    vec("enc.conv2.b", De)
    s.append(TensorSpec("enc.pos", (d.n_audio_ctx, De), F32, "sinusoid"))
    for i in range(d.n_audio_layer):
        p = f"enc.l{i}"
        ln(p + ".ln1", De)
        mat(p + ".qkv.w", (3 * De, De))
        vec(p + ".qkv.b", 3 * De, zero=(De, 2 * De))
        mat(p + ".o.w", (De, De))
        vec(p + ".o.b", De)
        ln(p + ".ln2", De)
        mat(p + ".fc1.w", (4 * De, De))
        vec(p + ".fc1.b", 4 * De)
        mat(p + ".fc2.w", (De, 4 * De))
        vec(p + ".fc2.b", De)
    ln("enc.lnpost", De)

    mat("dec.tok", (d.n_vocab, Dd), emb_std * u)
    vec("dec.pos", d.n_text_ctx * Dd, pos_std * u)
    L = d.n_text_layer
    mat("dec.crosskv.w", (L * 2 * Dd, De))
    # per layer: [k bias (zero) | v bias]
    s.append(TensorSpec("dec.crosskv.b", (L * 2 * Dd,), F32, "uniform", B))
    for i in range(L):
        p = f"dec.l{i}"
        ln(p + ".ln1", Dd)
        mat(p + ".qkv.w", (3 * Dd, Dd))
        vec(p + ".qkv.b", 3 * Dd, zero=(Dd, 2 * Dd))
        mat(p + ".o.w", (Dd, Dd))
        vec(p + ".o.b", Dd)
        ln(p + ".ln2", Dd)
        mat(p + ".xq.w", (Dd, Dd))
        vec(p + ".xq.b", Dd)
        mat(p + ".xo.w", (Dd, Dd))
        vec(p + ".xo.b", Dd)
        ln(p + ".ln3", Dd)
        mat(p + ".fc1.w", (4 * Dd, Dd))
        vec(p + ".fc1.b", 4 * Dd)
        mat(p + ".fc2.w", (Dd, 4 * Dd))
        vec(p + ".fc2.b", Dd)
    vec("dec.lnpost.g", Dd, G * out_gain, out_gain)
    vec("dec.lnpost.b", Dd, B)
    return s


def spec_shape(spec: TensorSpec, d: WhisperDims) -> tuple:
    if spec.name == "dec.pos":
        return (d.n_text_ctx, d.n_text_state)
    return spec.shape


# --------------------------------------------------------------------------
# counter-based hash init (mirrors osw_init_uniform in csrc/kernels_misc.hip)
# --------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def stream_key(seed: int, stream: int) -> int:
    k = _splitmix64(np.array([(seed * 0x632BE59BD9B4E019 + stream * 0x2545F4914F6CDD1D)
                              & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))
    return int(k[0])


def hash_uniform(seed: int, stream: int, n: int, scale: float, offset: float) -> np.ndarray:
    """x[i] = (2·u_i − 1)·scale + offset in fp32, u_i = top 24 bits of splitmix64(key + i) / 2^24."""
    key = np.uint64(stream_key(seed, stream))
    out = np.empty(n, dtype=np.float32)
    chunk = 1 << 22
    sc = np.float32(scale)
    of = np.float32(offset)
    with np.errstate(over="ignore"):
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            idx = np.arange(lo, hi, dtype=np.uint64) + key
            h = _splitmix64(idx)
            u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
            v = (u * np.float32(2.0) - np.float32(1.0)) * sc
            out[lo:hi] = v + of
    return out


def hash_uniform_at(seed: int, stream: int, idx: np.ndarray, scale: float, offset: float) -> np.ndarray:
    """The elements ``idx`` of ``hash_uniform(seed, stream, ...)`` (same values)."""
    key = np.uint64(stream_key(seed, stream))
    with np.errstate(over="ignore"):
        h = _splitmix64(np.asarray(idx, dtype=np.uint64) + key)
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (u * np.float32(2.0) - np.float32(1.0)) * np.float32(scale) + np.float32(offset)


TEXT_TS_AMP = 0.6     # weight of the timestamp target relative to the text target


def text_targets(d: WhisperDims, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """The two target tokens of every decoder position (``text_positional``): a
    pseudo-random text token below <|endoftext|>, and a timestamp token that rises
    with the position (first ones <= 1.00 s, as the initial-timestamp rule requires)."""
    from .dims import SpecialTokens
    st = SpecialTokens.for_vocab(d.n_vocab)
    n = d.n_text_ctx
    v = hash_uniform(seed, 9002, n, 0.5, 0.5).astype(np.float64)
    text = np.minimum((v * st.eot).astype(np.int64), st.eot - 1)
    ts = st.timestamp_begin + np.minimum((np.arange(n) * 1400) // n, 1500)
    return text, ts


def text_positional(d: WhisperDims, seed: int, amp: float, noise: float = 1.0, **spec_kw) -> np.ndarray:
    """A decoder positional table that makes greedy decoding of random weights emit
    varied text with clear top-2 margins (the "text" goldens, tools/make_golden.py):
    pos[p] = amp * (tok[text(p)] + TEXT_TS_AMP * tok[ts(p)]) + uniform noise of std
    ``noise``, where tok is the (fp16) token-embedding table of
    ``random_weights(d, seed, **spec_kw)`` and text(p) / ts(p) the position's targets
    (``text_targets``).  With the tied output projection the hidden state at position
    p leans towards text(p), and towards ts(p) where the timestamp rules force a
    timestamp, so ids change every step and rule-forced steps are not near-ties (the
    i.i.d. default init decodes near-ties between thousands of tokens, or timestamp
    pairs and a handful of repeated tokens).  The rest of the model is unchanged."""
    specs = canonical_specs(d, **spec_kw)
    i_tok = next(i for i, sp in enumerate(specs) if sp.name == "dec.tok")
    D = d.n_text_state
    text, ts = text_targets(d, seed)

    def rows(t):
        idx = (t[:, None] * D + np.arange(D)[None, :]).reshape(-1)
        return hash_uniform_at(seed, i_tok, idx, specs[i_tok].scale, 0.0).astype(np.float16).astype(np.float32)

    nz = hash_uniform(seed, 9003, d.n_text_ctx * D, noise * math.sqrt(3.0), 0.0)
    x = np.float32(amp) * (rows(text) + np.float32(TEXT_TS_AMP) * rows(ts)) + nz
    return x.reshape(d.n_text_ctx, D).astype(np.float32)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> np.ndarray:
    """Encoder positional table (openai-whisper ``sinusoids``; transformers
    modeling_whisper.py:55).  Real checkpoints store this table; random init regenerates it."""
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = np.exp(-inc * np.arange(channels // 2, dtype=np.float64))
    t = np.arange(length, dtype=np.float64)[:, None] * inv[None, :]
    return np.concatenate([np.sin(t), np.cos(t)], axis=1).astype(np.float32)


def make_tensor(spec: TensorSpec, d: WhisperDims, seed: int, stream: int) -> np.ndarray:
    shape = spec_shape(spec, d)
    if spec.kind == "sinusoid":
        return sinusoids(shape[0], shape[1])
    x = hash_uniform(seed, stream, spec.numel, spec.scale, spec.offset)
    if spec.zero_hi > spec.zero_lo:
        x[spec.zero_lo:spec.zero_hi] = 0.0
    if spec.name == "dec.crosskv.b":  # k-bias blocks are zero
        Dd = d.n_text_state
        x = x.reshape(d.n_text_layer, 2, Dd)
        x[:, 0, :] = 0.0
        x = x.reshape(-1)
    x = x.reshape(shape)
    return x.astype(np.float16) if spec.dtype == F16 else x


def random_weights(d: WhisperDims, seed: int = 0, text_pos: float | None = None, **kw) -> dict[str, np.ndarray]:
    """The canonical hash-initialised weights; ``text_pos`` (an amplitude): the decoder
    positional table of ``text_positional`` instead of the i.i.d. one."""
    w = {sp.name: make_tensor(sp, d, seed, i) for i, sp in enumerate(canonical_specs(d, **kw))}
    if text_pos:
        w["dec.pos"] = text_positional(d, seed, text_pos, **kw)
    return w


# --------------------------------------------------------------------------
# HuggingFace transformers Whisper state-dict <-> canonical
# --------------------------------------------------------------------------
def to_hf_state_dict(w: dict[str, np.ndarray], d: WhisperDims) -> dict[str, np.ndarray]:
    """Canonical -> transformers WhisperForConditionalGeneration names (fp32)."""
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    De, Dd = d.n_audio_state, d.n_text_state
    sd = {}
    sd["model.encoder.conv1.weight"] = f(w["enc.conv1.w"].transpose(0, 2, 1))
    sd["model.encoder.conv1.bias"] = f(w["enc.conv1.b"])
    sd["model.encoder.conv2.weight"] = f(w["enc.conv2.w"].transpose(0, 2, 1))
    sd["model.encoder.conv2.bias"] = f(w["enc.conv2.b"])
    sd["model.encoder.embed_positions.weight"] = f(w["enc.pos"])
    for i in range(d.n_audio_layer):
        p, q = f"enc.l{i}", f"model.encoder.layers.{i}"
        qkv, b = w[p + ".qkv.w"], w[p + ".qkv.b"]
        for j, nm in enumerate("qkv"):
            sd[f"{q}.self_attn.{nm}_proj.weight"] = f(qkv[j * De:(j + 1) * De])
            if nm != "k":
                sd[f"{q}.self_attn.{nm}_proj.bias"] = f(b[j * De:(j + 1) * De])
        sd[f"{q}.self_attn.out_proj.weight"] = f(w[p + ".o.w"])
        sd[f"{q}.self_attn.out_proj.bias"] = f(w[p + ".o.b"])
        sd[f"{q}.self_attn_layer_norm.weight"] = f(w[p + ".ln1.g"])
        sd[f"{q}.self_attn_layer_norm.bias"] = f(w[p + ".ln1.b"])
        sd[f"{q}.final_layer_norm.weight"] = f(w[p + ".ln2.g"])
        sd[f"{q}.final_layer_norm.bias"] = f(w[p + ".ln2.b"])
        for nm in ("fc1", "fc2"):
            sd[f"{q}.{nm}.weight"] = f(w[f"{p}.{nm}.w"])
            sd[f"{q}.{nm}.bias"] = f(w[f"{p}.{nm}.b"])
    sd["model.encoder.layer_norm.weight"] = f(w["enc.lnpost.g"])
    sd["model.encoder.layer_norm.bias"] = f(w["enc.lnpost.b"])
    sd["model.decoder.embed_tokens.weight"] = f(w["dec.tok"])
    sd["proj_out.weight"] = f(w["dec.tok"])
    sd["model.decoder.embed_positions.weight"] = f(w["dec.pos"])
    kv, kvb = w["dec.crosskv.w"], w["dec.crosskv.b"]
    for i in range(d.n_text_layer):
        p, q = f"dec.l{i}", f"model.decoder.layers.{i}"
        qkv, b = w[p + ".qkv.w"], w[p + ".qkv.b"]
        for j, nm in enumerate("qkv"):
            sd[f"{q}.self_attn.{nm}_proj.weight"] = f(qkv[j * Dd:(j + 1) * Dd])
            if nm != "k":
                sd[f"{q}.self_attn.{nm}_proj.bias"] = f(b[j * Dd:(j + 1) * Dd])
        sd[f"{q}.self_attn.out_proj.weight"] = f(w[p + ".o.w"])
        sd[f"{q}.self_attn.out_proj.bias"] = f(w[p + ".o.b"])
        sd[f"{q}.encoder_attn.q_proj.weight"] = f(w[p + ".xq.w"])
        sd[f"{q}.encoder_attn.q_proj.bias"] = f(w[p + ".xq.b"])
        base = i * 2 * Dd
        sd[f"{q}.encoder_attn.k_proj.weight"] = f(kv[base:base + Dd])
        sd[f"{q}.encoder_attn.v_proj.weight"] = f(kv[base + Dd:base + 2 * Dd])
        sd[f"{q}.encoder_attn.v_proj.bias"] = f(kvb[base + Dd:base + 2 * Dd])
        sd[f"{q}.encoder_attn.out_proj.weight"] = f(w[p + ".xo.w"])
        sd[f"{q}.encoder_attn.out_proj.bias"] = f(w[p + ".xo.b"])
        for a, c in (("ln1", "self_attn_layer_norm"), ("ln2", "encoder_attn_layer_norm"),
                     ("ln3", "final_layer_norm")):
            sd[f"{q}.{c}.weight"] = f(w[f"{p}.{a}.g"])
            sd[f"{q}.{c}.bias"] = f(w[f"{p}.{a}.b"])
        for nm in ("fc1", "fc2"):
            sd[f"{q}.{nm}.weight"] = f(w[f"{p}.{nm}.w"])
            sd[f"{q}.{nm}.bias"] = f(w[f"{p}.{nm}.b"])
    sd["model.decoder.layer_norm.weight"] = f(w["dec.lnpost.g"])
    sd["model.decoder.layer_norm.bias"] = f(w["dec.lnpost.b"])
    return sd


def from_hf_state_dict(sd: dict, d: WhisperDims) -> dict[str, np.ndarray]:
    """transformers Whisper state dict (numpy or torch tensors) -> canonical layout."""
    def g(k):
        v = sd[k]
        if hasattr(v, "detach"):
            v = v.detach().float().cpu().numpy()
        return np.asarray(v, dtype=np.float32)

    h16 = lambda a: np.ascontiguousarray(a, dtype=np.float16)  # noqa: E731
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    De, Dd = d.n_audio_state, d.n_text_state
    w = {}
    w["enc.conv1.w"] = h16(g("model.encoder.conv1.weight").transpose(0, 2, 1))
    w["enc.conv1.b"] = f32(g("model.encoder.conv1.bias"))
    w["enc.conv2.w"] = h16(g("model.encoder.conv2.weight").transpose(0, 2, 1))
    w["enc.conv2.b"] = f32(g("model.encoder.conv2.bias"))
    w["enc.pos"] = f32(g("model.encoder.embed_positions.weight"))

    def bias_or_zero(k, n):
        return g(k) if k in sd else np.zeros(n, np.float32)

    for i in range(d.n_audio_layer):
        p, q = f"enc.l{i}", f"model.encoder.layers.{i}"
        w[p + ".qkv.w"] = h16(np.concatenate([g(f"{q}.self_attn.{n}_proj.weight") for n in "qkv"]))
        w[p + ".qkv.b"] = f32(np.concatenate([bias_or_zero(f"{q}.self_attn.{n}_proj.bias", De)
                                              if n != "k" else np.zeros(De, np.float32) for n in "qkv"]))
        w[p + ".o.w"] = h16(g(f"{q}.self_attn.out_proj.weight"))
        w[p + ".o.b"] = f32(g(f"{q}.self_attn.out_proj.bias"))
        w[p + ".ln1.g"] = f32(g(f"{q}.self_attn_layer_norm.weight"))
        w[p + ".ln1.b"] = f32(g(f"{q}.self_attn_layer_norm.bias"))
        w[p + ".ln2.g"] = f32(g(f"{q}.final_layer_norm.weight"))
        w[p + ".ln2.b"] = f32(g(f"{q}.final_layer_norm.bias"))
        for nm in ("fc1", "fc2"):
            w[f"{p}.{nm}.w"] = h16(g(f"{q}.{nm}.weight"))
            w[f"{p}.{nm}.b"] = f32(g(f"{q}.{nm}.bias"))
    w["enc.lnpost.g"] = f32(g("model.encoder.layer_norm.weight"))
    w["enc.lnpost.b"] = f32(g("model.encoder.layer_norm.bias"))
    w["dec.tok"] = h16(g("model.decoder.embed_tokens.weight"))
    w["dec.pos"] = f32(g("model.decoder.embed_positions.weight"))
    kv, kvb = [], []
    for i in range(d.n_text_layer):
        p, q = f"dec.l{i}", f"model.decoder.layers.{i}"
        w[p + ".qkv.w"] = h16(np.concatenate([g(f"{q}.self_attn.{n}_proj.weight") for n in "qkv"]))
        w[p + ".qkv.b"] = f32(np.concatenate([bias_or_zero(f"{q}.self_attn.{n}_proj.bias", Dd)
                                              if n != "k" else np.zeros(Dd, np.float32) for n in "qkv"]))
        w[p + ".o.w"] = h16(g(f"{q}.self_attn.out_proj.weight"))
        w[p + ".o.b"] = f32(g(f"{q}.self_attn.out_proj.bias"))
        w[p + ".xq.w"] = h16(g(f"{q}.encoder_attn.q_proj.weight"))
        w[p + ".xq.b"] = f32(g(f"{q}.encoder_attn.q_proj.bias"))
        w[p + ".xo.w"] = h16(g(f"{q}.encoder_attn.out_proj.weight"))
        w[p + ".xo.b"] = f32(g(f"{q}.encoder_attn.out_proj.bias"))
        kv += [g(f"{q}.encoder_attn.k_proj.weight"), g(f"{q}.encoder_attn.v_proj.weight")]
        kvb += [np.zeros(Dd, np.float32), bias_or_zero(f"{q}.encoder_attn.v_proj.bias", Dd)]
        for a, c in (("ln1", "self_attn_layer_norm"), ("ln2", "encoder_attn_layer_norm"),
                     ("ln3", "final_layer_norm")):
            w[f"{p}.{a}.g"] = f32(g(f"{q}.{c}.weight"))
            w[f"{p}.{a}.b"] = f32(g(f"{q}.{c}.bias"))
        for nm in ("fc1", "fc2"):
            w[f"{p}.{nm}.w"] = h16(g(f"{q}.{nm}.weight"))
            w[f"{p}.{nm}.b"] = f32(g(f"{q}.{nm}.bias"))
    w["dec.crosskv.w"] = h16(np.concatenate(kv))
    w["dec.crosskv.b"] = f32(np.concatenate(kvb))
    w["dec.lnpost.g"] = f32(g("model.decoder.layer_norm.weight"))
    w["dec.lnpost.b"] = f32(g("model.decoder.layer_norm.bias"))
    return w


def dims_from_hf_config(cfg: dict) -> WhisperDims:
    return WhisperDims(n_mels=cfg["num_mel_bins"], n_audio_ctx=cfg.get("max_source_positions", 1500),
                       n_audio_state=cfg["d_model"], n_audio_head=cfg["encoder_attention_heads"],
                       n_audio_layer=cfg["encoder_layers"], n_vocab=cfg["vocab_size"],
                       n_text_ctx=cfg.get("max_target_positions", 448), n_text_state=cfg["d_model"],
                       n_text_head=cfg["decoder_attention_heads"], n_text_layer=cfg["decoder_layers"])
