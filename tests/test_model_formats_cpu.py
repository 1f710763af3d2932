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
