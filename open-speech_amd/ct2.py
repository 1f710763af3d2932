"""CTranslate2 ``model.bin`` reader (and a writer for tests) for Whisper checkpoints.

The reference's default model (``STT_MODEL=deepdml/faster-whisper-large-v3-turbo-ct2``,
``src/config.py:141``) is a CTranslate2 directory: ``model.bin`` + ``config.json`` +
``tokenizer.json`` (+ ``vocabulary.json``, ``preprocessor_config.json``).

Binary layout restated from CTranslate2's public spec serializer
(``ctranslate2/specs/model_spec.py`` ``_serialize``; upstream, not vendored, no real
file available offline — the round trip below is self-consistent, parity against a
real file is unverified):

    u32 version | str spec_name | u32 revision | u32 n_vars
    n_vars x { str name | u8 rank | rank x u32 dim | u8 dtype | u32 nbytes | bytes }
    u32 n_aliases | n_aliases x { str alias | str target }
    str = u16 length (incl. NUL) | utf-8 bytes | NUL

dtype ids: 0 float32, 1 int8, 2 int16, 3 int32, 4 float16, 5 bfloat16.  int8 weights
carry a per-row ``<name>_scale`` (float32) variable; they are dequantised here.

Variable names (CTranslate2 ``WhisperSpec`` as produced by its transformers
converter): ``encoder/conv1/weight`` ``[D, n_mels, 3]``; ``encoder/layer_i/
self_attention/linear_0`` = fused q|k|v (k bias 0); ``linear_1`` = out-proj;
``ffn/linear_0|1``; ``decoder/layer_i/attention/linear_0`` = cross q,
``linear_1`` = fused cross k|v, ``linear_2`` = cross out; layer norms are
``gamma``/``beta``; ``decoder/embeddings/weight``; ``*/position_encodings/encodings``.
"""
from __future__ import annotations

import struct

import numpy as np

from .dims import WhisperDims

_DT = {0: np.float32, 1: np.int8, 2: np.int16, 3: np.int32, 4: np.float16}
_DT_ID = {np.dtype(np.float32): 0, np.dtype(np.int8): 1, np.dtype(np.int16): 2, np.dtype(np.int32): 3,
          np.dtype(np.float16): 4}


def _bf16_to_f32(raw: bytes, shape) -> np.ndarray:
    u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
    return u.view(np.float32).reshape(shape)


def read_model_bin(path: str) -> tuple[dict, dict]:
    """Returns (variables name -> ndarray, aliases alias -> target)."""
    with open(path, "rb") as fh:
        buf = fh.read()
    off = 0

    def u(fmt):
        nonlocal off
        v = struct.unpack_from("<" + fmt, buf, off)[0]
        off += struct.calcsize(fmt)
        return v

    def string():
        nonlocal off
        n = u("H")
        s = buf[off:off + n - 1].decode("utf-8")
        off += n
        return s

    version = u("I")
    if version < 2 or version > 6:
        raise ValueError(f"unsupported CTranslate2 binary version {version}")
    string()            # spec name
    if version >= 3:
        u("I")          # revision
    nvar = u("I")
    vars_: dict = {}
    for _ in range(nvar):
        name = string()
        rank = u("B")
        shape = tuple(u("I") for _ in range(rank))
        if version >= 4:
            dt = u("B")
            nbytes = u("I")
        else:  # v2/v3: item size then count
            item = u("B")
            count = u("I")
            dt = {4: 0, 1: 1, 2: 2}.get(item, 0)
            nbytes = item * count
        raw = buf[off:off + nbytes]
        off += nbytes
        if dt == 5:
            arr = _bf16_to_f32(raw, shape)
        else:
            arr = np.frombuffer(raw, dtype=_DT[dt]).reshape(shape)
        vars_[name] = arr
    aliases = {}
    if off < len(buf):
        for _ in range(u("I")):
            a = string()
            aliases[a] = string()
    return vars_, aliases


def write_model_bin(path: str, variables: dict, aliases: dict | None = None, spec: str = "WhisperSpec") -> None:
    def s(x: str) -> bytes:
        b = x.encode("utf-8")
        return struct.pack("<H", len(b) + 1) + b + b"\0"

    with open(path, "wb") as fh:
        fh.write(struct.pack("<I", 6) + s(spec) + struct.pack("<I", 3) + struct.pack("<I", len(variables)))
        for name, arr in variables.items():
            a = np.ascontiguousarray(arr)
            fh.write(s(name) + struct.pack("<B", a.ndim) + b"".join(struct.pack("<I", d) for d in a.shape))
            fh.write(struct.pack("<B", _DT_ID[a.dtype]) + struct.pack("<I", a.nbytes) + a.tobytes())
        aliases = aliases or {}
        fh.write(struct.pack("<I", len(aliases)))
        for a, t in aliases.items():
            fh.write(s(a) + s(t))


def _get(v: dict, aliases: dict, name: str) -> np.ndarray:
    name = aliases.get(name, name)
    if name not in v:
        raise ValueError(f"CTranslate2 model.bin has no variable {name!r}, which the Whisper spec requires "
                         f"(found {len(v)} variables, e.g. {sorted(v)[:3]})")
    x = v[name]
    sc = v.get(name + "_scale")
    if x.dtype == np.int8 and sc is not None:  # per-row int8 quantisation
        x = x.astype(np.float32) / np.asarray(sc, np.float32).reshape(-1, *([1] * (x.ndim - 1)))
    return np.asarray(x, dtype=np.float32)


def dims_from_ct2(v: dict) -> WhisperDims:
    for k in ("encoder/conv1/weight", "decoder/embeddings/weight", "decoder/position_encodings/encodings",
              "encoder/position_encodings/encodings"):
        if k not in v:
            raise ValueError(f"not a CTranslate2 Whisper model.bin: no {k!r}")
    D, n_mels, _ = v["encoder/conv1/weight"].shape
    import re

    n_enc = len({m.group(1) for k in v if (m := re.match(r"encoder/layer_(\d+)/", k))})
    n_dec = len({m.group(1) for k in v if (m := re.match(r"decoder/layer_(\d+)/", k))})
    V = v["decoder/embeddings/weight"].shape[0]
    ctx = v["decoder/position_encodings/encodings"].shape[0]
    return WhisperDims(n_mels=n_mels, n_audio_ctx=v["encoder/position_encodings/encodings"].shape[0],
                       n_audio_state=D, n_audio_head=D // 64, n_audio_layer=n_enc, n_vocab=V, n_text_ctx=ctx,
                       n_text_state=D, n_text_head=D // 64, n_text_layer=n_dec)


def ct2_to_canonical(v: dict, aliases: dict, d: WhisperDims) -> dict:
    g = lambda n: _get(v, aliases, n)  # noqa: E731
    h16 = lambda a: np.ascontiguousarray(a, dtype=np.float16)  # noqa: E731
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    w = {}
    w["enc.conv1.w"] = h16(g("encoder/conv1/weight").transpose(0, 2, 1))
    w["enc.conv1.b"] = f32(g("encoder/conv1/bias"))
    w["enc.conv2.w"] = h16(g("encoder/conv2/weight").transpose(0, 2, 1))
    w["enc.conv2.b"] = f32(g("encoder/conv2/bias"))
    w["enc.pos"] = f32(g("encoder/position_encodings/encodings"))
    for i in range(d.n_audio_layer):
        p, q = f"enc.l{i}", f"encoder/layer_{i}"
        w[p + ".ln1.g"] = f32(g(f"{q}/self_attention/layer_norm/gamma"))
        w[p + ".ln1.b"] = f32(g(f"{q}/self_attention/layer_norm/beta"))
        w[p + ".qkv.w"] = h16(g(f"{q}/self_attention/linear_0/weight"))
        w[p + ".qkv.b"] = f32(g(f"{q}/self_attention/linear_0/bias"))
        w[p + ".o.w"] = h16(g(f"{q}/self_attention/linear_1/weight"))
        w[p + ".o.b"] = f32(g(f"{q}/self_attention/linear_1/bias"))
        w[p + ".ln2.g"] = f32(g(f"{q}/ffn/layer_norm/gamma"))
        w[p + ".ln2.b"] = f32(g(f"{q}/ffn/layer_norm/beta"))
        w[p + ".fc1.w"] = h16(g(f"{q}/ffn/linear_0/weight"))
        w[p + ".fc1.b"] = f32(g(f"{q}/ffn/linear_0/bias"))
        w[p + ".fc2.w"] = h16(g(f"{q}/ffn/linear_1/weight"))
        w[p + ".fc2.b"] = f32(g(f"{q}/ffn/linear_1/bias"))
    w["enc.lnpost.g"] = f32(g("encoder/layer_norm/gamma"))
    w["enc.lnpost.b"] = f32(g("encoder/layer_norm/beta"))
    w["dec.tok"] = h16(g("decoder/embeddings/weight"))
    w["dec.pos"] = f32(g("decoder/position_encodings/encodings"))
    kv, kvb = [], []
    for i in range(d.n_text_layer):
        p, q = f"dec.l{i}", f"decoder/layer_{i}"
        w[p + ".ln1.g"] = f32(g(f"{q}/self_attention/layer_norm/gamma"))
        w[p + ".ln1.b"] = f32(g(f"{q}/self_attention/layer_norm/beta"))
        w[p + ".qkv.w"] = h16(g(f"{q}/self_attention/linear_0/weight"))
        w[p + ".qkv.b"] = f32(g(f"{q}/self_attention/linear_0/bias"))
        w[p + ".o.w"] = h16(g(f"{q}/self_attention/linear_1/weight"))
        w[p + ".o.b"] = f32(g(f"{q}/self_attention/linear_1/bias"))
        w[p + ".ln2.g"] = f32(g(f"{q}/attention/layer_norm/gamma"))
        w[p + ".ln2.b"] = f32(g(f"{q}/attention/layer_norm/beta"))
        w[p + ".xq.w"] = h16(g(f"{q}/attention/linear_0/weight"))
        w[p + ".xq.b"] = f32(g(f"{q}/attention/linear_0/bias"))
        kv.append(g(f"{q}/attention/linear_1/weight"))
        kvb.append(g(f"{q}/attention/linear_1/bias"))
        w[p + ".xo.w"] = h16(g(f"{q}/attention/linear_2/weight"))
        w[p + ".xo.b"] = f32(g(f"{q}/attention/linear_2/bias"))
        w[p + ".ln3.g"] = f32(g(f"{q}/ffn/layer_norm/gamma"))
        w[p + ".ln3.b"] = f32(g(f"{q}/ffn/layer_norm/beta"))
        w[p + ".fc1.w"] = h16(g(f"{q}/ffn/linear_0/weight"))
        w[p + ".fc1.b"] = f32(g(f"{q}/ffn/linear_0/bias"))
        w[p + ".fc2.w"] = h16(g(f"{q}/ffn/linear_1/weight"))
        w[p + ".fc2.b"] = f32(g(f"{q}/ffn/linear_1/bias"))
    w["dec.crosskv.w"] = h16(np.concatenate(kv))
    w["dec.crosskv.b"] = f32(np.concatenate(kvb))
    w["dec.lnpost.g"] = f32(g("decoder/layer_norm/gamma"))
    w["dec.lnpost.b"] = f32(g("decoder/layer_norm/beta"))
    return w


def canonical_to_ct2(w: dict, d: WhisperDims, dtype=np.float16) -> tuple[dict, dict]:
    """Inverse mapping (test fixture writer): canonical tensors -> CT2 variable dict."""
    c = lambda a: np.ascontiguousarray(a, dtype=dtype)  # noqa: E731
    f = lambda a: np.ascontiguousarray(a, dtype=np.float32)  # noqa: E731
    v = {"encoder/conv1/weight": c(w["enc.conv1.w"].transpose(0, 2, 1)), "encoder/conv1/bias": f(w["enc.conv1.b"]),
         "encoder/conv2/weight": c(w["enc.conv2.w"].transpose(0, 2, 1)), "encoder/conv2/bias": f(w["enc.conv2.b"]),
         "encoder/position_encodings/encodings": f(w["enc.pos"])}
    for i in range(d.n_audio_layer):
        p, q = f"enc.l{i}", f"encoder/layer_{i}"
        v[f"{q}/self_attention/layer_norm/gamma"] = f(w[p + ".ln1.g"])
        v[f"{q}/self_attention/layer_norm/beta"] = f(w[p + ".ln1.b"])
        v[f"{q}/self_attention/linear_0/weight"] = c(w[p + ".qkv.w"])
        v[f"{q}/self_attention/linear_0/bias"] = f(w[p + ".qkv.b"])
        v[f"{q}/self_attention/linear_1/weight"] = c(w[p + ".o.w"])
        v[f"{q}/self_attention/linear_1/bias"] = f(w[p + ".o.b"])
        v[f"{q}/ffn/layer_norm/gamma"] = f(w[p + ".ln2.g"])
        v[f"{q}/ffn/layer_norm/beta"] = f(w[p + ".ln2.b"])
        v[f"{q}/ffn/linear_0/weight"] = c(w[p + ".fc1.w"])
        v[f"{q}/ffn/linear_0/bias"] = f(w[p + ".fc1.b"])
        v[f"{q}/ffn/linear_1/weight"] = c(w[p + ".fc2.w"])
        v[f"{q}/ffn/linear_1/bias"] = f(w[p + ".fc2.b"])
    v["encoder/layer_norm/gamma"] = f(w["enc.lnpost.g"])
    v["encoder/layer_norm/beta"] = f(w["enc.lnpost.b"])
    v["decoder/embeddings/weight"] = c(w["dec.tok"])
    v["decoder/position_encodings/encodings"] = f(w["dec.pos"])
    Dd = d.n_text_state
    for i in range(d.n_text_layer):
        p, q = f"dec.l{i}", f"decoder/layer_{i}"
        v[f"{q}/self_attention/layer_norm/gamma"] = f(w[p + ".ln1.g"])
        v[f"{q}/self_attention/layer_norm/beta"] = f(w[p + ".ln1.b"])
        v[f"{q}/self_attention/linear_0/weight"] = c(w[p + ".qkv.w"])
        v[f"{q}/self_attention/linear_0/bias"] = f(w[p + ".qkv.b"])
        v[f"{q}/self_attention/linear_1/weight"] = c(w[p + ".o.w"])
        v[f"{q}/self_attention/linear_1/bias"] = f(w[p + ".o.b"])
        v[f"{q}/attention/layer_norm/gamma"] = f(w[p + ".ln2.g"])
        v[f"{q}/attention/layer_norm/beta"] = f(w[p + ".ln2.b"])
        v[f"{q}/attention/linear_0/weight"] = c(w[p + ".xq.w"])
        v[f"{q}/attention/linear_0/bias"] = f(w[p + ".xq.b"])
        v[f"{q}/attention/linear_1/weight"] = c(w["dec.crosskv.w"][i * 2 * Dd:(i + 1) * 2 * Dd])
        v[f"{q}/attention/linear_1/bias"] = f(w["dec.crosskv.b"][i * 2 * Dd:(i + 1) * 2 * Dd])
        v[f"{q}/attention/linear_2/weight"] = c(w[p + ".xo.w"])
        v[f"{q}/attention/linear_2/bias"] = f(w[p + ".xo.b"])
        v[f"{q}/ffn/layer_norm/gamma"] = f(w[p + ".ln3.g"])
        v[f"{q}/ffn/layer_norm/beta"] = f(w[p + ".ln3.b"])
        v[f"{q}/ffn/linear_0/weight"] = c(w[p + ".fc1.w"])
        v[f"{q}/ffn/linear_0/bias"] = f(w[p + ".fc1.b"])
        v[f"{q}/ffn/linear_1/weight"] = c(w[p + ".fc2.w"])
        v[f"{q}/ffn/linear_1/bias"] = f(w[p + ".fc2.b"])
    v["decoder/layer_norm/gamma"] = f(w["dec.lnpost.g"])
    v["decoder/layer_norm/beta"] = f(w["dec.lnpost.b"])
    return v, {"decoder/projection/weight": "decoder/embeddings/weight"}
