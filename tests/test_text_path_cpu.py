"""The text path with a real ``tokenizer.json``: tokenizer decode,
``initial_prompt`` encoding into the decoder prefix, the tokenizer-derived non-speech
set, ``compression_ratio`` and the response shapes on real text.

The tokenizer is the synthetic Whisper-layout byte-level BPE of ``tests/tokfix.py``
(no Whisper tokenizer exists offline); the engine is the scripted stand-in of
``test_backend_cpu.py``, so these run without a GPU.  What they pin is faster-whisper
1.2.1's host-side semantics (upstream, not vendored): ``Tokenizer.decode`` keeps ids
< eot; ``non_speech_tokens`` / ``get_suppressed_tokens``; the prompt
``[<|startofprev|>] + encode(" " + initial_prompt.strip()) + previous text``; segment
text = decode(segment tokens); ``compression_ratio`` = len(utf-8) / len(zlib) of the
window's decoded text, stripped; ``avg_logprob`` = sum_logprob / (n + 1)."""
import json
import zlib

import numpy as np
import pytest

import tokfix
from open_speech_amd import dims as D
from open_speech_amd import synth
from open_speech_amd.engine import WindowOutput
from open_speech_amd.tokenizer import _MISC, _SYMBOLS, WhisperTokenizer, compression_ratio, get_suppressed_tokens
from test_backend_cpu import make_backend

ST = D.SpecialTokens.for_vocab(51866)
TB = ST.timestamp_begin


@pytest.fixture(scope="module")
def tok_path(tmp_path_factory):
    return tokfix.build_tokenizer_json(str(tmp_path_factory.mktemp("tok") / "tokenizer.json"))


@pytest.fixture(scope="module")
def model_dir(tmp_path_factory):
    return tokfix.make_hf_model_dir(str(tmp_path_factory.mktemp("micro_hf")), D.MICRO_TEST)


def test_tokenizer_layout_and_decode(tok_path):
    tk = WhisperTokenizer(51866, tok_path)
    assert tk.has_text
    raw = tk._tok
    assert raw.get_vocab_size() == 51866
    assert raw.token_to_id("<|endoftext|>") == ST.eot and raw.token_to_id("<|startoftranscript|>") == ST.sot
    assert raw.token_to_id("<|en|>") == ST.first_lang and raw.token_to_id("<|transcribe|>") == ST.transcribe
    assert raw.token_to_id("<|startofprev|>") == ST.sot_prev and raw.token_to_id("<|notimestamps|>") == ST.no_timestamps
    assert raw.token_to_id("<|0.00|>") == TB and raw.token_to_id("<|30.00|>") == 51865
    for line in tokfix.CORPUS:
        ids = tk.encode(" " + line)
        assert all(0 <= t < ST.eot for t in ids)
        assert tk.decode(ids) == " " + line
        # decode keeps text ids only (faster-whisper Tokenizer.decode: token < eot)
        assert tk.decode([TB] + ids + [TB + 7, ST.eot]) == " " + line
    assert tk.decode([40000]) == " zq40000"


def test_non_speech_tokens_from_tokenizer(tok_path):
    """faster-whisper's rule: encode(" -")[0], encode(" '")[0], and every symbol whose
    encoding (bare or space-prefixed) is ONE token; the music symbols' first token
    always.  suppress_tokens=[-1] = that set + the task / sot / prev / lm specials."""
    tk = WhisperTokenizer(51866, tok_path)
    raw = tk._tok
    want = {raw.encode(" -", add_special_tokens=False).ids[0], raw.encode(" '", add_special_tokens=False).ids[0]}
    for sym in _SYMBOLS + sorted(_MISC):
        for s in (sym, " " + sym):
            ids = raw.encode(s, add_special_tokens=False).ids
            if len(ids) == 1 or sym in _MISC:
                want.add(ids[0])
    got = tk.non_speech_tokens()
    assert got == tuple(sorted(want))
    assert len(got) > 20
    # the trained merges made some multi-character symbols single tokens: they are in
    assert any(len(raw.encode(s, add_special_tokens=False).ids) == 1 and raw.encode(s, add_special_tokens=False).ids[0]
               in got for s in ("--", "[[", "<<"))
    sup = get_suppressed_tokens(tk, [-1])
    assert sup == tuple(sorted(set(got) | {ST.transcribe, ST.translate, ST.sot, ST.sot_prev, ST.sot_lm}))
    assert get_suppressed_tokens(tk, [5, 7]) == tuple(sorted({5, 7, ST.transcribe, ST.translate, ST.sot, ST.sot_prev,
                                                               ST.sot_lm}))


def test_compression_ratio_on_text():
    t = "Hello world. " * 30
    b = t.encode("utf-8")
    assert compression_ratio(t) == len(b) / len(zlib.compress(b))
    assert compression_ratio(t) > 2.4                    # the faster-whisper repetition threshold
    assert compression_ratio("") == 0.0


def _script(tk):
    """Window 0: two timestamped segments then an unfinished third (seek moves to the
    last timestamp); later windows: one segment that ends the window."""
    a, b = tk.encode(" Hello world."), tk.encode(" The quick brown fox.")
    c = tk.encode(" Whisper transcribes speech into text with timestamps.")

    def script(w, i, prefix, lang):
        if w[1] == 0:                      # the window at seek 0
            return WindowOutput([TB] + a + [TB + 150, TB + 150] + b + [TB + 400, TB + 400] + c, -4.0, 0.01,
                                ST.first_lang)
        return WindowOutput([TB] + c + [TB + 500], -3.0, 0.02, ST.first_lang)
    return script


def test_backend_text_fields_and_prompt(model_dir):
    """verbose_json through HipWhisperBackend with a model directory carrying
    tokenizer.json: segment texts are the tokenizer's decode of their tokens, the
    window text's compression ratio and avg_logprob are faster-whisper's, the
    initial prompt is encoded into the first window's prefix and later windows are
    conditioned on the previous segments' tokens."""
    tk = WhisperTokenizer(51866, model_dir + "/tokenizer.json")
    holder = []
    be = make_backend(_script(tk), holder)
    prompt = "  Meeting notes: budget review. "
    res = be.transcribe(audio=synth.to_wav_bytes(synth.chirp_clip(0, 45.0)), model=model_dir,
                        response_format="verbose_json", prompt=prompt)
    eng = holder[0]
    segs = res["segments"]
    assert [s["text"] for s in segs[:2]] == [" Hello world.", " The quick brown fox."]
    for s in segs:
        assert s["text"] == tk.decode(s["tokens"])
    # window 0: the decoded window text (all its tokens), stripped
    toks0 = [TB] + tk.encode(" Hello world.") + [TB + 150, TB + 150] + tk.encode(" The quick brown fox.") + \
        [TB + 400, TB + 400] + tk.encode(" Whisper transcribes speech into text with timestamps.")
    text0 = tk.decode(toks0).strip().encode("utf-8")
    assert segs[0]["compression_ratio"] == len(text0) / len(zlib.compress(text0))
    assert segs[0]["avg_logprob"] == pytest.approx(-4.0 / (len(toks0) + 1))
    assert res["text"] == "".join(s["text"] for s in segs).strip()
    # prompts: window 0 = [sot_prev] + encode(" " + prompt.strip()); window 1 adds the
    # tokens of window 0's kept segments (condition_on_previous_text)
    init = tk.encode(" " + prompt.strip())
    (w0win, pre0, _, _), (w1win, pre1, _, _) = eng.calls[0], eng.calls[1]
    assert pre0 == [ST.sot_prev] + init
    kept = [t for s in segs if s["seek"] == 0 for t in s["tokens"]]
    assert pre1 == [ST.sot_prev] + (init + kept)[-(448 // 2 - 1):]
    # window 1 starts at window 0's last complete timestamp pair: 8.00 s -> frame 800
    assert w1win[1] == 800
    # text / srt shapes on the same text
    txt = be.transcribe(audio=synth.to_wav_bytes(synth.chirp_clip(0, 45.0)), model=model_dir,
                        response_format="text", prompt=prompt)
    assert txt == {"text": res["text"], "raw_text": True}
    srt = be.transcribe(audio=synth.to_wav_bytes(synth.chirp_clip(0, 45.0)), model=model_dir,
                        response_format="srt", prompt=prompt)["text"]
    assert srt.startswith("1\n00:00:00,000 --> 00:00:03,000\nHello world.\n")
    be.unload_model(model_dir)


def test_backend_without_prompt_has_no_prefix(model_dir):
    tk = WhisperTokenizer(51866, model_dir + "/tokenizer.json")
    holder = []
    be = make_backend(_script(tk), holder)
    be.transcribe(audio=synth.to_wav_bytes(synth.chirp_clip(1, 20.0)), model=model_dir,
                  response_format="json")
    assert holder[0].calls[0][1] == []
    be.unload_model(model_dir)


def test_hf_model_dir_resolves_tokenizer(model_dir):
    from open_speech_amd import model_store
    src = model_store.resolve(model_dir)
    assert src.kind == "hf" and src.tokenizer_json and src.dims == D.MICRO_TEST
    w = model_store.load_weights(src)
    assert w["dec.tok"].shape == (51866, 128)
    with open(model_dir + "/config.json") as fh:
        assert json.load(fh)["vocab_size"] == 51866
    assert np.isfinite(w["dec.lnpost.g"]).all()
