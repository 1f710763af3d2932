#!/usr/bin/env python3
"""Pin the oracle's long-form seek loop (oracle/seek.py, faster-whisper's
``generate_segments`` restated) against transformers' own long-form sequential
generation (``WhisperGenerationMixin.generate``, models/whisper/generation_whisper.py:
383-968; run here, on CPU; writes tests/golden/hf_longform_pin.npz + a meta entry).

Both sides decode the same 75 s clip with the same tiny-test hash weights, temperature
0, condition on previous text, no-speech threshold 0.6, log-prob threshold -1, no
compression-ratio threshold, timestamps on, max_length 448, language <|en|>.  The
model's logits carry the position-scheduled bias of tests/hf_longform_pin.py so the
transcript takes the loop's branches (timestamp pairs, single endings, partial-window
seeks, <|endoftext|> and max_length windows).  Where the two loops coincide and where
they differ:

* window cut: faster-whisper's ``content_frames = n_frames - 1`` of the 160-sample-padded
  whole-file log-mel; transformers loops while ``seek < total_input_frames``.  The log-mel
  handed to transformers is therefore the oracle's without its last frame; both pad a
  window to 3000 frames with zeros.
* previous-text prompt: ``[<|startofprev|>] + last 223 tokens`` of the earlier segments in
  both; transformers drops the closing timestamp of a segment that ends in a timestamp
  pair (``skip_ending_double_timestamps``), which is exactly faster-whisper's segment
  (it slices that pair apart).  faster-whisper also drops segments with start == end or
  blank text from the prompt; transformers keeps them: the generator asserts no such
  segment occurs (the comparison's precondition).
* segments: transformers' last segment of a window that ends in a timestamp pair keeps
  both timestamps; the comparison drops the second one (faster-whisper's slice).
* skip rule: no_speech_prob > 0.6 and avg log-prob below -1 (transformers: strictly
  below; faster-whisper: not above; equal only at the threshold).

The generator runs the oracle's ``seek_loop`` with transformers' (biased) decoder
(``make_golden._HFStepper``) and asserts that its segments equal transformers', then
stores transformers' segments; tests/test_oracle_hf_longform.py replays the oracle's
numpy model (fp32) against them.

Usage:  python tools/make_hf_longform_pin.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import make_golden as mg  # noqa: E402
from hf_longform_pin import bias_row  # noqa: E402

from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth, weights  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402
from oracle import decode as odec  # noqa: E402
from oracle import seek as oseek  # noqa: E402

from transformers import GenerationConfig, WhisperForConditionalGeneration  # noqa: E402

SEED = 1234
EMB_STD = 0.1
CLIP = 21
SECONDS = 75.0


class Biased(WhisperForConditionalGeneration):
    """transformers' Whisper with tests/hf_longform_pin.py's bias added to the logits of
    every decoder position (the position = the self-attention cache length before the
    call + the token's index in it)."""

    st = None

    def forward(self, *a, **kw):
        past = kw.get("past_key_values")
        p0 = past.get_seq_length() if past is not None else 0
        o = super().forward(*a, **kw)
        T = o.logits.shape[1]
        bias = np.stack([bias_row(p0 + i, self.st, o.logits.shape[-1]) for i in range(T)])
        o.logits = o.logits + torch.from_numpy(bias)[None].to(o.logits.dtype)
        return o


def hf_generation_config(st, sup):
    return GenerationConfig(decoder_start_token_id=st.sot, eos_token_id=st.eot, pad_token_id=st.eot,
                            no_timestamps_token_id=st.no_timestamps, prev_sot_token_id=st.sot_prev,
                            is_multilingual=True, lang_to_id={"<|en|>": st.first_lang},
                            task_to_id={"transcribe": st.transcribe, "translate": st.translate},
                            begin_suppress_tokens=[st.blank, st.eot], suppress_tokens=list(sup),
                            max_initial_timestamp_index=50, max_length=448, return_timestamps=True)


def hf_segments(model, mel, st, sup):
    """transformers' long-form result as (start, end, tokens) in faster-whisper's slicing."""
    gc = hf_generation_config(st, sup)
    model.generation_config = gc
    feats = torch.from_numpy(np.ascontiguousarray(mel[:, :mel.shape[1] - 1]))[None]
    out = model.generate(input_features=feats, attention_mask=torch.ones(1, feats.shape[-1], dtype=torch.long),
                         generation_config=gc, language="en", task="transcribe", return_timestamps=True,
                         condition_on_prev_tokens=True, temperature=0.0, logprob_threshold=-1.0,
                         no_speech_threshold=0.6, compression_ratio_threshold=None, return_segments=True)
    segs = []
    for s in out["segments"][0]:
        toks = s["tokens"].tolist()
        if len(toks) > 2 and toks[-2] >= st.timestamp_begin and toks[-1] >= st.timestamp_begin:
            toks = toks[:-1]   # the closing timestamp of a pair belongs to the next slice
        segs.append((float(s["start"]), float(s["end"]), toks))
    return segs


def oracle_segments(stepper_for_window, n_frames, st, sup):
    """oracle.seek.seek_loop with the oracle's greedy window decoder over a stepper."""
    opts = odec.DecodeOptions(suppress_tokens=sup)

    def decode_window(seek, size, prompt):
        orc = stepper_for_window(seek, size)
        r = odec.greedy_from_encoder(orc, None, st, language=st.first_lang,
                                     prev_tokens=prompt[1:] if prompt else (), opts=opts)
        return r.tokens, r.sum_logprob, r.no_speech_prob

    wins = oseek.seek_loop(decode_window, n_frames, st, lambda t: "x")
    return wins, [(a, b, t) for w in wins for a, b, t in w.segments]


def window_mel(mel, seek, size):
    x = np.zeros((mel.shape[0], 3000), np.float32)
    x[:, :size] = mel[:, seek:seek + size]
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    a = ap.parse_args()
    torch.manual_seed(0)
    d = D.TINY_TEST
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=SEED, emb_std=EMB_STD)
    base = mg.build_model(d, w)
    Biased.st = st
    model = Biased(base.config).eval()
    model.load_state_dict(base.state_dict())
    pcm = synth.chirp_clip(CLIP, SECONDS)
    mel = mg.fe_mel(pcm, d.n_mels)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    hf = hf_segments(model, mel, st, sup)

    def stepper(seek, size):
        with torch.no_grad():
            enc = model.model.encoder(input_features=torch.from_numpy(window_mel(mel, seek, size))[None])
        return mg._HFStepper(model, enc.last_hidden_state)

    wins, mine = oracle_segments(stepper, mel.shape[1], st, sup)
    assert all(a != b for a, b, _ in hf), "a start == end segment: faster-whisper would drop it from the prompt"
    assert len(mine) == len(hf), (len(mine), len(hf))
    for (a0, b0, t0), (a1, b1, t1) in zip(mine, hf):
        assert t0 == t1 and abs(a0 - a1) < 1e-6 and abs(b0 - b1) < 1e-6, ((a0, b0, t0), (a1, b1, t1))
    for s in hf:
        print(round(s[0], 2), round(s[1], 2), s[2][:10], len(s[2]))
    print("windows", [(w.seek, w.size, len(w.prompt), len(w.tokens), w.skipped) for w in wins])
    flat = [t for _, _, toks in hf for t in toks]
    np.savez_compressed(os.path.join(a.out, "hf_longform_pin.npz"), starts=np.array([s[0] for s in hf]),
                        ends=np.array([s[1] for s in hf]), lens=np.array([len(s[2]) for s in hf], np.int32),
                        ids=np.array(flat, np.int32))
    mp = os.path.join(a.out, "meta.json")
    m = json.load(open(mp)) if os.path.exists(mp) else {}
    m["hf_longform_pin"] = {"generator": "tools/make_hf_longform_pin.py", "seed": SEED, "emb_std": EMB_STD,
                            "clip": CLIP, "seconds": SECONDS, "n_segments": len(hf),
                            "windows": [[w.seek, w.size, len(w.prompt), len(w.tokens), w.skipped] for w in wins]}
    with open(mp, "w") as fh:
        json.dump(m, fh, indent=1)


if __name__ == "__main__":
    main()
