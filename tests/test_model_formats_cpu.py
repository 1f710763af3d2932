"""On-disk model formats (no GPU): CTranslate2 model.bin round trip, HF safetensors
directory, and model-id resolution through the cache layout the reference scans
(src/backends/faster_whisper.py:93-208)."""
import json

import numpy as np
import pytest

from open_speech_amd import ct2, model_store, weights
from open_speech_amd import dims as D

d = D.MICRO_TEST


@pytest.fixture(scope="module")
def canon():
    return weights.random_weights(d, seed=3)


def _eq(a, b):
    for k in a:
        assert a[k].dtype == b[k].dtype, k
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_ct2_roundtrip(tmp_path, canon):
    v, al = ct2.canonical_to_ct2(canon, d)
    p = tmp_path / "model.bin"
    ct2.write_model_bin(str(p), v, al)
    v2, al2 = ct2.read_model_bin(str(p))
    assert al2 == al and set(v2) == set(v)
    assert ct2.dims_from_ct2(v2) == d
    _eq(canon, ct2.ct2_to_canonical(v2, al2, d))


def test_ct2_int8_dequant(tmp_path, canon):
    v, al = ct2.canonical_to_ct2(canon, d, dtype=np.float32)
    w = v["encoder/layer_0/ffn/linear_0/weight"]
    scale = 127.0 / np.abs(w).max(axis=1)
    v["encoder/layer_0/ffn/linear_0/weight"] = np.round(w * scale[:, None]).astype(np.int8)
    v["encoder/layer_0/ffn/linear_0/weight_scale"] = scale.astype(np.float32)
    p = tmp_path / "model.bin"
    ct2.write_model_bin(str(p), v, al)
    v2, al2 = ct2.read_model_bin(str(p))
    out = ct2.ct2_to_canonical(v2, al2, d)["enc.l0.fc1.w"].astype(np.float32)
    np.testing.assert_allclose(out, w, atol=np.abs(w).max() / 127 + 1e-3)


def test_hf_safetensors_and_resolution(tmp_path, canon):
    from safetensors.numpy import save_file
    snap = tmp_path / "models--org--tiny-whisper" / "snapshots" / "abc"
    snap.mkdir(parents=True)
    sd = {k: v.astype(np.float16) for k, v in weights.to_hf_state_dict(canon, d).items() if k != "proj_out.weight"}
    save_file(sd, str(snap / "model.safetensors"))
    cfg = {"num_mel_bins": d.n_mels, "d_model": d.n_audio_state, "encoder_attention_heads": d.n_audio_head,
           "encoder_layers": d.n_audio_layer, "decoder_attention_heads": d.n_text_head,
           "decoder_layers": d.n_text_layer, "vocab_size": d.n_vocab}
    (snap / "config.json").write_text(json.dumps(cfg))
    src = model_store.resolve("org/tiny-whisper", str(tmp_path))
    assert src.kind == "hf" and src.dims == d
    w = model_store.load_weights(src)
    for k in canon:
        np.testing.assert_allclose(w[k].astype(np.float32), canon[k].astype(np.float32), atol=2e-3, err_msg=k)


def test_ct2_directory_resolution(tmp_path, canon):
    snap = tmp_path / "models--deepdml--faster-whisper-micro-ct2" / "snapshots" / "x"
    snap.mkdir(parents=True)
    v, al = ct2.canonical_to_ct2(canon, d)
    ct2.write_model_bin(str(snap / "model.bin"), v, al)
    src = model_store.resolve("deepdml/faster-whisper-micro-ct2", str(tmp_path))
    assert src.kind == "ct2" and src.dims == d
    _eq(canon, model_store.load_weights(src))


def test_random_and_missing():
    assert model_store.resolve("random:tiny-test:7").seed == 7
    with pytest.raises(FileNotFoundError):
        model_store.resolve("nobody/nothing", "/nonexistent-dir")


def test_ct2_hand_built_v6_header(tmp_path):
    """A model.bin written byte by byte from CTranslate2's published serializer layout
    (ctranslate2/specs/model_spec.py _serialize, version 6; upstream, not vendored):
    the reader does not depend on this package's own writer.  Includes an int8 weight
    with its per-row float32 ``<name>_scale`` (CT2 quantises q = round(w * scale),
    scale = 127 / max|w_row|, so w = q / scale) and an alias entry."""
    import struct

    def s(x):
        b = x.encode()
        return struct.pack("<H", len(b) + 1) + b + b"\0"

    q = np.array([[127, -64], [10, -127]], np.int8)
    sc = np.array([127 / 2.0, 127 / 0.5], np.float32)
    bias = np.array([0.25, -1.5], np.float32)
    buf = struct.pack("<I", 6) + s("WhisperSpec") + struct.pack("<I", 3) + struct.pack("<I", 3)
    for name, arr, dt in (("decoder/layer_0/ffn/linear_0/weight", q, 1),
                          ("decoder/layer_0/ffn/linear_0/weight_scale", sc, 0),
                          ("decoder/layer_0/ffn/linear_0/bias", bias, 0)):
        buf += s(name) + struct.pack("<B", arr.ndim) + b"".join(struct.pack("<I", x) for x in arr.shape)
        buf += struct.pack("<B", dt) + struct.pack("<I", arr.nbytes) + arr.tobytes()
    buf += struct.pack("<I", 1) + s("decoder/projection/weight") + s("decoder/embeddings/weight")
    p = tmp_path / "model.bin"
    p.write_bytes(buf)
    v, al = ct2.read_model_bin(str(p))
    assert al == {"decoder/projection/weight": "decoder/embeddings/weight"}
    assert v["decoder/layer_0/ffn/linear_0/weight"].dtype == np.int8
    w = ct2._get(v, al, "decoder/layer_0/ffn/linear_0/weight")
    np.testing.assert_allclose(w, q / sc[:, None], rtol=1e-7)
    with pytest.raises(ValueError, match="decoder/layer_0/ffn/linear_1/weight"):
        ct2._get(v, al, "decoder/layer_0/ffn/linear_1/weight")
    with pytest.raises(ValueError, match="not a CTranslate2 Whisper"):
        ct2.dims_from_ct2(v)


def test_ct2_whisper_variable_names(canon):
    """The CT2 WhisperSpec names the converter writes for one encoder / decoder layer
    (the fused self-attention q|k|v is linear_0 with a zero k bias; cross-attention is
    linear_0 = q, linear_1 = fused k|v, linear_2 = out).  ASSUMPTION (parity unpinned:
    no real CT2 file offline): CT2 applies 1/sqrt(head_dim) inside its attention, so the
    stored query weights are the checkpoint's unscaled q_proj."""
    v, al = ct2.canonical_to_ct2(canon, d)
    want = {"encoder/layer_0/self_attention/linear_0/weight", "encoder/layer_0/self_attention/linear_1/weight",
            "encoder/layer_0/self_attention/layer_norm/gamma", "encoder/layer_0/ffn/linear_0/weight",
            "encoder/layer_0/ffn/linear_1/weight", "encoder/layer_0/ffn/layer_norm/beta",
            "decoder/layer_0/attention/linear_0/weight", "decoder/layer_0/attention/linear_1/weight",
            "decoder/layer_0/attention/linear_2/weight", "decoder/layer_0/self_attention/linear_0/bias",
            "decoder/embeddings/weight", "decoder/position_encodings/encodings", "encoder/conv1/weight",
            "encoder/conv2/bias", "encoder/layer_norm/gamma", "decoder/layer_norm/beta"}
    assert want <= set(v)
    D_ = d.n_text_state
    assert v["decoder/layer_0/attention/linear_1/weight"].shape == (2 * D_, D_)
    assert not v["encoder/layer_0/self_attention/linear_0/bias"][D_:2 * D_].any()   # k bias zero
