"""Test fixtures for the text path: a synthetic Whisper-layout byte-level BPE
``tokenizer.json`` and a transformers-layout model directory around it.

No Whisper tokenizer file exists offline, so the tokenizer is built
here with the ``tokenizers`` package (importable on both machines): a byte-level BPE
trained on a small fixed corpus (it merges words and some of faster-whisper's
non-speech symbols into single tokens), padded with filler tokens to the 50257 text
ids of the multilingual vocabulary, followed by Whisper's special tokens at their ids
(``<|endoftext|>`` 50257 ... ``<|notimestamps|>`` 50364, ``<|0.00|>`` 50365 ...
``<|30.00|>`` 51865).  Every id a random-weight decoder can emit therefore decodes.
The file is generated into a temporary directory per test session, deterministically
from this module; it is test data, not product code.
"""
from __future__ import annotations

import json
import os

CORPUS = [
    "Hello world. This is a test of the transcription path.",
    "The quick brown fox jumps over the lazy dog, again and again.",
    "She said -- quietly -- that the meeting (the second one) was cancelled.",
    "Numbers like 42 and 1999; times like 10:30 and 22:15.",
    "[[inline]] ((double)) <<quoted>> and -- dashes -- everywhere.",
    "Whisper transcribes speech into text with timestamps.",
    "Don't stop: it's only the beginning, isn't it?",
    "A music note ♪ may appear, and then ♪♪ two of them.",
]


def build_tokenizer_json(path: str, n_vocab: int = 51866) -> str:
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    import osw_path
    osw_path.load()
    from open_speech_amd.dims import LANGUAGE_CODES, SpecialTokens

    st = SpecialTokens.for_vocab(n_vocab)
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=700, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                             show_progress=False)
    tok.train_from_iterator(CORPUS * 40, tr)
    s = json.loads(tok.to_str())
    vocab = s["model"]["vocab"]
    base = len(vocab)
    assert base < st.eot
    for i in range(base, st.eot):          # filler text tokens: id i decodes to " zq<i>"
        vocab[f"Ġzq{i}"] = i
    specials = (["<|endoftext|>", "<|startoftranscript|>"]
                + [f"<|{c}|>" for c in LANGUAGE_CODES[:st.n_langs]]
                + ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nospeech|>",
                   "<|notimestamps|>"]
                + [f"<|{i * 0.02:.2f}|>" for i in range(n_vocab - st.timestamp_begin)])
    assert st.eot + len(specials) == n_vocab
    s["added_tokens"] = [{"id": st.eot + k, "content": t, "single_word": False, "lstrip": False, "rstrip": False,
                          "normalized": False, "special": True} for k, t in enumerate(specials)]
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(s, fh, ensure_ascii=False)
    return path


def make_hf_model_dir(root: str, dims, seed: int = 7, emb_std: float = 0.5) -> str:
    """config.json + model.safetensors (random weights at `dims`, transformers names) +
    the synthetic tokenizer.json: what model_store resolves as an "hf" checkpoint."""
    import numpy as np
    from safetensors.numpy import save_file

    import osw_path
    osw_path.load()
    from open_speech_amd import weights

    os.makedirs(root, exist_ok=True)
    cfg = {"model_type": "whisper", "num_mel_bins": dims.n_mels, "max_source_positions": dims.n_audio_ctx,
           "d_model": dims.n_audio_state, "encoder_attention_heads": dims.n_audio_head,
           "encoder_layers": dims.n_audio_layer, "vocab_size": dims.n_vocab,
           "max_target_positions": dims.n_text_ctx, "decoder_attention_heads": dims.n_text_head,
           "decoder_layers": dims.n_text_layer}
    with open(os.path.join(root, "config.json"), "w") as fh:
        json.dump(cfg, fh)
    w = weights.random_weights(dims, seed=seed, emb_std=emb_std)
    sd = {k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.to_hf_state_dict(w, dims).items()}
    save_file(sd, os.path.join(root, "model.safetensors"))
    build_tokenizer_json(os.path.join(root, "tokenizer.json"), dims.n_vocab)
    return root
