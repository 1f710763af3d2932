#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run here, on CPU; committed).

The reference (faster-whisper 1.2.1 + CTranslate2) is not installed and cannot be
fetched, and the reference's own tests pin no numbers for this path.
The fixtures therefore come from an independent implementation of the same
published algorithm that IS in the image: transformers 5.15.0
(``WhisperFeatureExtractor``, ``WhisperForConditionalGeneration`` in fp32, and its
Whisper logits processors), with random weights from the canonical hash init so
that tests can regenerate the weights instead of storing them.

Usage:  python tools/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth, weights  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

from transformers import GenerationConfig, WhisperConfig, WhisperFeatureExtractor  # noqa: E402
from transformers import WhisperForConditionalGeneration  # noqa: E402
from transformers.generation.logits_process import (  # noqa: E402
    SuppressTokensAtBeginLogitsProcessor, SuppressTokensLogitsProcessor,
    WhisperTimeStampLogitsProcessor)

TINY_SEED = 1234
TINY_EMB_STD = 0.5
TURBO_LAYER_SEED = 77


def hf_config(d: D.WhisperDims) -> WhisperConfig:
    return WhisperConfig(vocab_size=d.n_vocab, num_mel_bins=d.n_mels, encoder_layers=d.n_audio_layer,
                         encoder_attention_heads=d.n_audio_head, decoder_layers=d.n_text_layer,
                         decoder_attention_heads=d.n_text_head, d_model=d.n_audio_state,
                         encoder_ffn_dim=4 * d.n_audio_state, decoder_ffn_dim=4 * d.n_text_state,
                         max_source_positions=d.n_audio_ctx, max_target_positions=d.n_text_ctx,
                         pad_token_id=50257, bos_token_id=50257, eos_token_id=50257,
                         decoder_start_token_id=50258, attn_implementation="eager")


def fe_mel(pcm: np.ndarray, n_mels: int) -> np.ndarray:
    """transformers' extractor applied to faster-whisper's 160-sample-padded waveform."""
    fe = WhisperFeatureExtractor(feature_size=n_mels)
    x = pcm.astype(np.float32) / 32768.0
    x = np.pad(x, (0, 160))
    return fe._np_extract_fbank_features(x[None, :], "cpu")[0].astype(np.float32)


def gen_mel(out):
    clips = {
        "chirp30": (synth.chirp_clip(0, 30.0), 128),
        "tone7": (synth.tone_clip(7.3), 80),
        "silence5": (synth.silence_clip(5.0), 128),
        "chirp3": (synth.chirp_clip(5, 3.21), 80),
    }
    meta = {}
    for name, (pcm, n_mels) in clips.items():
        mel = fe_mel(pcm, n_mels)
        np.savez_compressed(os.path.join(out, f"mel_{name}.npz"), pcm=pcm, mel=mel,
                            n_mels=np.int32(n_mels))
        meta[name] = {"n_samples": int(len(pcm)), "n_mels": n_mels, "frames": int(mel.shape[1]),
                      "pcm_sha256": hashlib.sha256(pcm.tobytes()).hexdigest()}
        print("mel", name, mel.shape)
    return meta


def build_model(d: D.WhisperDims, w: dict):
    model = WhisperForConditionalGeneration(hf_config(d)).eval()
    sd = {k: torch.from_numpy(v) for k, v in weights.to_hf_state_dict(w, d).items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [m for m in missing if not m.endswith("k_proj.bias")]
    assert not missing and not unexpected, (missing, unexpected)
    return model


def gen_tiny(out):
    d = D.TINY_TEST
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=TINY_SEED, emb_std=TINY_EMB_STD)
    model = build_model(d, w)
    pcm = synth.chirp_clip(3, 30.0)
    mel = fe_mel(pcm, d.n_mels)[:, :3000]
    with torch.no_grad():
        enc = model.model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
    tok = WhisperTokenizer(d.n_vocab)
    suppress = get_suppressed_tokens(tok, [-1])
    gc = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                          max_initial_timestamp_index=50)

    def step(ids, past):
        with torch.no_grad():
            o = model(encoder_outputs=(enc,), decoder_input_ids=torch.tensor([ids]), past_key_values=past,
                      use_cache=True)
        return o.logits[0, -1].float(), o.past_key_values

    lg, past = step([st.sot], None)
    sot_logits = lg.numpy().copy()
    lang = st.first_lang + int(np.argmax(sot_logits[st.first_lang:st.first_lang + st.n_langs]))
    nsp = float(torch.softmax(lg.double(), -1)[st.no_speech])
    prompt = [st.sot, lang, st.transcribe]
    lg, past = step([lang], past)
    lg, past = step([st.transcribe], past)
    begin = len(prompt)
    procs = [SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], begin),
             SuppressTokensLogitsProcessor(list(suppress)),
             WhisperTimeStampLogitsProcessor(gc, begin)]
    seq = list(prompt)
    ids, lps, top5i, top5v, raw = [], [], [], [], []
    sum_lp = 0.0
    while True:
        if len(raw) < 8:
            raw.append(lg.numpy().copy())
        x = lg[None].clone()
        for p in procs:
            x = p(torch.tensor([seq]), x)
        lsm = torch.log_softmax(x.double(), -1)[0]
        nxt = int(torch.argmax(x[0]))
        v, i = torch.topk(lg, 5)
        top5i.append(i.numpy())
        top5v.append(v.numpy())
        sum_lp += float(lsm[nxt])
        lps.append(float(lsm[nxt]))
        if nxt == st.eot:
            break
        ids.append(nxt)
        seq.append(nxt)
        if len(seq) >= d.n_text_ctx:
            break
        lg, past = step([nxt], past)
    np.savez_compressed(os.path.join(out, "tiny_model.npz"), mel=mel, enc=enc[0].numpy().astype(np.float16),
                        sot_logits=sot_logits, step_logits=np.stack(raw), ids=np.array(ids, np.int32),
                        logprobs=np.array(lps), top5_ids=np.stack(top5i).astype(np.int32),
                        top5_vals=np.stack(top5v), language=np.int32(lang), no_speech_prob=np.float64(nsp),
                        sum_logprob=np.float64(sum_lp))
    print("tiny: lang", lang, "n_ids", len(ids), "first", ids[:12])
    return {"seed": TINY_SEED, "emb_std": TINY_EMB_STD, "language": lang, "n_ids": len(ids)}


def gen_turbo_layer(out):
    """Encoder layer 0 at whisper-large-v3-turbo dims (fp32, transformers)."""
    d = D.LARGE_V3_TURBO
    specs = weights.canonical_specs(d)
    idx = {s.name: i for i, s in enumerate(specs)}
    w = {}
    for nm in ("ln1.g", "ln1.b", "qkv.w", "qkv.b", "o.w", "o.b", "ln2.g", "ln2.b", "fc1.w", "fc1.b",
               "fc2.w", "fc2.b"):
        full = "enc.l0." + nm
        w[full] = weights.make_tensor(specs[idx[full]], d, TURBO_LAYER_SEED, idx[full])
    x = weights.hash_uniform(4242, 0, 1500 * 1280, 1.0, 0.0).reshape(1500, 1280)
    from transformers.models.whisper.modeling_whisper import WhisperEncoderLayer
    layer = WhisperEncoderLayer(hf_config(d)).eval()
    De = d.n_audio_state
    f = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    with torch.no_grad():
        sa = layer.self_attn
        qkv, b = w["enc.l0.qkv.w"], w["enc.l0.qkv.b"]
        sa.q_proj.weight.copy_(f(qkv[:De])); sa.q_proj.bias.copy_(f(b[:De]))
        sa.k_proj.weight.copy_(f(qkv[De:2 * De]))
        sa.v_proj.weight.copy_(f(qkv[2 * De:])); sa.v_proj.bias.copy_(f(b[2 * De:]))
        sa.out_proj.weight.copy_(f(w["enc.l0.o.w"])); sa.out_proj.bias.copy_(f(w["enc.l0.o.b"]))
        layer.self_attn_layer_norm.weight.copy_(f(w["enc.l0.ln1.g"]))
        layer.self_attn_layer_norm.bias.copy_(f(w["enc.l0.ln1.b"]))
        layer.final_layer_norm.weight.copy_(f(w["enc.l0.ln2.g"]))
        layer.final_layer_norm.bias.copy_(f(w["enc.l0.ln2.b"]))
        layer.fc1.weight.copy_(f(w["enc.l0.fc1.w"])); layer.fc1.bias.copy_(f(w["enc.l0.fc1.b"]))
        layer.fc2.weight.copy_(f(w["enc.l0.fc2.w"])); layer.fc2.bias.copy_(f(w["enc.l0.fc2.b"]))
        y = layer(torch.from_numpy(x)[None], attention_mask=None)
        y = (y[0] if isinstance(y, tuple) else y)[0].numpy()
    rows = np.r_[0:48, 700:716, 1452:1500]
    np.savez_compressed(os.path.join(out, "turbo_enc_layer0.npz"), rows=rows, y_rows=y[rows].astype(np.float32),
                        y_rownorm=np.linalg.norm(y.astype(np.float64), axis=1), x_seed=np.int32(4242),
                        w_seed=np.int32(TURBO_LAYER_SEED))
    print("turbo layer: |y| mean", float(np.abs(y).mean()))
    return {"w_seed": TURBO_LAYER_SEED, "x_seed": 4242}


TURBO_SEED = 0          # the bench's init_random(seed=0) weights
TURBO_CLIP = 0          # synth.chirp_clip(0, 30 s)
TURBO_FULL_STEPS = 4    # full-vocabulary fp32 logits stored for the first steps
TURBO_FULL_STRIDE = 32  # ... and for every 32nd step after them
TURBO_SUBSET = 256      # per step: logits of the top-32 tokens and of a fixed token sample


def gen_turbo(out):
    """whisper-large-v3-turbo end to end in fp32 (transformers): the encoder output
    (selected rows + every row norm), the <|startoftranscript|> logits, and greedy
    decoding to <|endoftext|> or 448 positions with the openai / faster-whisper
    logits rules — ids, the chosen tokens' log-probs, top-5 per step, and per step
    the log-sum-exp plus the logits of the top-32 and of a fixed token sample (so a
    log-softmax check covers every step without storing 51866 floats per step)."""
    d = D.LARGE_V3_TURBO
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=TURBO_SEED)
    model = build_model(d, w)
    del w
    pcm = synth.chirp_clip(TURBO_CLIP, 30.0)
    mel = fe_mel(pcm, d.n_mels)[:, :3000]
    with torch.no_grad():
        enc = model.model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
    tok = WhisperTokenizer(d.n_vocab)
    suppress = get_suppressed_tokens(tok, [-1])
    gc = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                          max_initial_timestamp_index=50)

    def step(ids, past):
        with torch.no_grad():
            o = model(encoder_outputs=(enc,), decoder_input_ids=torch.tensor([ids]), past_key_values=past,
                      use_cache=True)
        return o.logits[0, -1].double(), o.past_key_values

    lg, past = step([st.sot], None)
    sot_logits = lg.float().numpy().copy()
    lang = st.first_lang + int(np.argmax(sot_logits[st.first_lang:st.first_lang + st.n_langs]))
    nsp = float(torch.softmax(lg, -1)[st.no_speech])
    prompt = [st.sot, lang, st.transcribe]
    lg, past = step([lang], past)
    lg, past = step([st.transcribe], past)
    begin = len(prompt)
    procs = [SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], begin),
             SuppressTokensLogitsProcessor(list(suppress)),
             WhisperTimeStampLogitsProcessor(gc, begin)]
    sample = np.sort(np.random.default_rng(2024).choice(d.n_vocab, TURBO_SUBSET, replace=False)).astype(np.int32)
    seq = list(prompt)
    ids, lps, top5i, top5v, full, lse, sub_i, sub_v, margins = [], [], [], [], [], [], [], [], []
    full_steps = []
    sum_lp = 0.0
    while True:
        raw = lg.float().numpy()
        step_i = len(lse)
        if step_i < TURBO_FULL_STEPS or step_i % TURBO_FULL_STRIDE == 0:
            full.append(raw.copy())
            full_steps.append(step_i)
        lse.append(float(torch.logsumexp(lg, -1)))
        t32 = np.argsort(-raw, kind="stable")[:32].astype(np.int32)
        sub_i.append(np.concatenate([t32, sample]))
        sub_v.append(raw[sub_i[-1]])
        x = lg[None].clone().float()
        for p in procs:
            x = p(torch.tensor([seq]), x)
        lsm = torch.log_softmax(x.double(), -1)[0]
        top2 = torch.topk(x[0], 2).values
        margins.append(float(top2[0] - top2[1]))
        nxt = int(torch.argmax(x[0]))
        v, i = torch.topk(lg.float(), 5)
        top5i.append(i.numpy())
        top5v.append(v.numpy())
        sum_lp += float(lsm[nxt])
        lps.append(float(lsm[nxt]))
        if nxt == st.eot:
            break
        ids.append(nxt)
        seq.append(nxt)
        if len(seq) >= d.n_text_ctx:
            break
        lg, past = step([nxt], past)
    e = enc[0].numpy()
    rows = np.r_[0:8, 700:708, 1492:1500]
    np.savez_compressed(os.path.join(out, "turbo_model.npz"), enc_rows=rows, enc=e[rows].astype(np.float32),
                        enc_rownorm=np.linalg.norm(e.astype(np.float64), axis=1), sot_logits=sot_logits,
                        full_logits=np.stack(full), full_steps=np.array(full_steps, np.int32), lse=np.array(lse), sub_ids=np.stack(sub_i), sub_vals=np.stack(sub_v),
                        ids=np.array(ids, np.int32), logprobs=np.array(lps), top5_ids=np.stack(top5i).astype(np.int32),
                        top5_vals=np.stack(top5v), margins=np.array(margins), language=np.int32(lang),
                        no_speech_prob=np.float64(nsp), sum_logprob=np.float64(sum_lp))
    print("turbo: lang", lang, "n_ids", len(ids), "first", ids[:12], "min margin", min(margins))
    return {"seed": TURBO_SEED, "clip": TURBO_CLIP, "language": lang, "n_ids": len(ids),
            "min_top2_margin": min(margins)}


TURBO_BEAM_MAX_LEN = 96   # prompt (3) + 93 sampled positions: random weights never emit <|endoftext|>


class _HFStepper:
    """The decoder-step interface of oracle.model.WhisperOracle (new_cache /
    decoder_step) over the fp32 transformers model, so oracle.decode.beam_from_encoder
    (the CTranslate2 BeamSearch restatement) runs on transformers' arithmetic."""

    def __init__(self, model, enc):
        self.model, self.enc = model, enc

    def new_cache(self):
        return {"past": None}

    def decoder_step(self, tok, pos, cache, xkv):
        with torch.no_grad():
            o = self.model(encoder_outputs=(self.enc,), decoder_input_ids=torch.tensor([[int(tok)]]),
                           past_key_values=cache["past"], use_cache=True)
        cache["past"] = o.past_key_values
        return o.logits[0, -1].float().numpy()


def gen_turbo_beam(out):
    """whisper-large-v3-turbo beam search width 5 (the reference's decoding,
    src/backends/faster_whisper.py:237) in fp32: the oracle's CTranslate2-BeamSearch
    restatement (oracle/decode.py beam_from_encoder, patience 1, length penalty 1,
    one hypothesis) driven by the transformers decoder on the same hash-initialised
    weights and clip as gen_turbo, to TURBO_BEAM_MAX_LEN positions.  Stores the best
    hypothesis' ids and raw cumulative log-prob, the language and no-speech prob."""
    from oracle import decode as odec

    d = D.LARGE_V3_TURBO
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=TURBO_SEED)
    model = build_model(d, w)
    del w
    pcm = synth.chirp_clip(TURBO_CLIP, 30.0)
    mel = fe_mel(pcm, d.n_mels)[:, :3000]
    with torch.no_grad():
        enc = model.model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    r = odec.beam_from_encoder(_HFStepper(model, enc), None, st,
                               opts=odec.DecodeOptions(suppress_tokens=sup, max_length=TURBO_BEAM_MAX_LEN),
                               beam=odec.BeamOptions(beam_size=5))
    np.savez_compressed(os.path.join(out, "turbo_beam5.npz"), ids=np.array(r.tokens, np.int32),
                        sum_logprob=np.float64(r.sum_logprob), language=np.int32(r.language),
                        no_speech_prob=np.float64(r.no_speech_prob), max_length=np.int32(TURBO_BEAM_MAX_LEN))
    print("turbo beam5: lang", r.language, "n_ids", len(r.tokens), "sum_lp", r.sum_logprob, "first", r.tokens[:12])
    return {"seed": TURBO_SEED, "clip": TURBO_CLIP, "beam_size": 5, "max_length": TURBO_BEAM_MAX_LEN,
            "n_ids": len(r.tokens), "language": int(r.language)}


# "text" goldens: weights whose greedy decoding emits varied text (weights.text_positional:
# the decoder positional table leans every position towards a pseudo-random target token),
# so an id check discriminates (the i.i.d. init above decodes timestamp pairs and a handful
# of repeated tokens: 10 distinct ids in 445).  The rest of the model is the default init.
#
# Round 6: with the positional lean alone the ids hardly depend on the
# audio (two of the old three clips gave identical ids, the third differed at 2 of 445), so a
# decoder whose cross-attention ignored the encoder would still pass.  The turbo table is
# now CONSTRUCTED (construct_audio_table): at most positions the lean is split between the
# target and a second token chosen so that the clips' own audio (through the cross-attention)
# decides between them, with a margin on every side.  The three clips are spectrally
# distinct (a chirp, a 440 Hz tone, white noise), and the generator asserts that every pair of
# clips differs at >= TEXT_MIN_PAIR_DIFF of the 445 ids.
TEXT_SEED = 11
TEXT_AMP = 20.0         # turbo: the base lean (min top-2 margin 0.04 over 3 x 445 steps, ~440 distinct ids per clip)
TINY_TEXT_AMP = 200.0   # tiny dims: the GPU's tiny encoder is held to 1e-2, so larger margins (min 1.4)
TEXT_CLIPS = {"chirp0": lambda: synth.chirp_clip(0, 30.0), "tone": lambda: synth.tone_clip(30.0),
              "noise": lambda: synth.noise_clip(5, 30.0)}
TEXT_SPLIT_MARGIN = 0.08    # top-2 margin of every clip at every split position (GPU logits error ~5e-4)
TEXT_MIN_PAIR_DIFF = 100    # ids that must differ between every pair of clips
TEXT_MAX_SHIFT = 8.0        # largest logit shift a split may need
TEXT_REPAIR_MARGIN = 0.12   # below this, a position's row is nudged to widen its smallest margin


def _rules(st, suppress):
    gc = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                          max_initial_timestamp_index=50)
    return [SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], 3),
            SuppressTokensLogitsProcessor(list(suppress)),
            WhisperTimeStampLogitsProcessor(gc, 3)]


def _apply_rules(procs, seq, logits):
    x = torch.from_numpy(np.asarray(logits, np.float32).copy())[None]
    for p in procs:
        x = p(torch.tensor([seq]), x)
    return x[0].double().numpy()


def _top2(x):
    i = np.argpartition(-x, 2)[:2]
    v = np.sort(x[i])[::-1]
    return float(v[0] - v[1])


def _log(*a):
    print(*a, flush=True)


def construct_audio_table(d, w, encs: dict, log=_log, split_margin=None, repair_margin=None):
    """Builds the decoder positional table of the "text" goldens so that the greedy ids
    depend on the audio.  Positions are built in order, on the fp32 oracle (oracle/model.py,
    fp16=False: transformers' arithmetic), all clips decoding side by side with their own
    caches and logits rules.  At input position q the base row is text_positional's.  When
    every clip's argmax is the same text token a, the generator looks for a second text token
    t whose logit gap to a, v_c = x_c[t] - x_c[a], varies across the clips through their
    audio, picks the largest gap between two clips' v, and adds beta * E[t] (E: the tied
    token embedding) to the row so that the middle of that gap lands on zero (secant on
    beta): the clips on one side of the gap emit t, the others a, each with top-2 margin
    >= split_margin (TEXT_SPLIT_MARGIN), else the position keeps its base row.  The isolated clip is chosen
    to balance the per-pair differences.  Returns (table, ids per clip, split count)."""
    from oracle.model import WhisperOracle

    split_margin = TEXT_SPLIT_MARGIN if split_margin is None else split_margin
    repair_margin = TEXT_REPAIR_MARGIN if repair_margin is None else repair_margin
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    suppress = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    procs = _rules(st, suppress)
    w = dict(w)
    w["dec.pos"] = np.array(w["dec.pos"], np.float32).reshape(d.n_text_ctx, d.n_text_state).copy()
    orc = WhisperOracle(d, w, fp16=False)
    table = orc.w["dec.pos"]
    E = orc.w["dec.tok"]
    names = list(encs)
    nc = len(names)
    xkv = {n: orc.cross_kv(encs[n]) for n in names}
    cache = {n: orc.new_cache() for n in names}
    seq, prev, ids = {}, {}, {n: [] for n in names}
    for n in names:
        lg = orc.decoder_step(st.sot, 0, cache[n], xkv[n])
        lang = st.first_lang + int(np.argmax(lg[st.first_lang:st.first_lang + st.n_langs]))
        orc.decoder_step(lang, 1, cache[n], xkv[n])
        seq[n], prev[n] = [st.sot, lang, st.transcribe], st.transcribe
    pairs = {(i, j): 0 for i in range(nc) for j in range(i + 1, nc)}

    def evaluate(row, q):
        table[q] = row
        return [_apply_rules(procs, seq[n], orc.decoder_step(prev[n], q, cache[n], xkv[n])) for n in names]

    n_split = n_repair = 0
    for q in range(2, d.n_text_ctx - 1):
        r0 = table[q].copy()
        xs = evaluate(r0, q)
        am = [int(np.argmax(x)) for x in xs]
        final = xs
        if len(set(am)) == 1 and am[0] < st.eot:
            a = am[0]
            X = np.stack(xs)
            ok = np.isfinite(X).all(0)
            ok[st.eot:] = False
            ok[a] = False
            cand = np.nonzero(ok)[0]
            v = X[:, cand] - X[:, a][:, None]
            order = np.argsort(v, axis=0)
            vs = np.take_along_axis(v, order, 0)
            low = min(pairs, key=pairs.get)             # the pair with the fewest differences
            best = None
            for k in range(nc - 1):                     # gap between sorted clips k and k+1
                gap = vs[k + 1] - vs[k]
                shift = -(vs[k] + vs[k + 1]) / 2.0
                # the clips below the gap keep a, the ones above switch to t
                for ci in np.nonzero((gap >= 2 * split_margin + 0.02) & (shift <= TEXT_MAX_SHIFT))[0]:
                    below = set(order[:k + 1, ci].tolist())
                    helps = (low[0] in below) != (low[1] in below)
                    score = gap[ci] * (1.0 if helps else 0.5)
                    if best is None or score > best[0]:
                        best = (score, int(cand[ci]), k, below, float(gap[ci]))
            if best is not None:
                _, t, k, below, gap = best
                lo_c, hi_c = [int(order[k, cand.tolist().index(t)]), int(order[k + 1, cand.tolist().index(t)])]

                def f(xl):
                    return 0.5 * ((xl[lo_c][t] - xl[lo_c][a]) + (xl[hi_c][t] - xl[hi_c][a]))
                b0, f0 = 0.0, f(xs)
                b1 = 4.0
                x1 = evaluate(r0 + np.float32(b1) * E[t], q)
                f1 = f(x1)
                for _ in range(4):
                    if not np.isfinite(f1) or abs(f1) < 0.1 * gap or f1 == f0:
                        break
                    b2 = b1 - f1 * (b1 - b0) / (f1 - f0)
                    b0, f0 = b1, f1
                    b1 = float(np.clip(b2, -200.0, 200.0))
                    x1 = evaluate(r0 + np.float32(b1) * E[t], q)
                    f1 = f(x1)
                am1 = [int(np.argmax(x)) for x in x1]
                want = [a if i in below else t for i in range(nc)]
                if np.isfinite(f1) and am1 == want and min(_top2(x) for x in x1) >= split_margin:
                    final = x1
                    n_split += 1
                else:
                    final = evaluate(r0, q)
        # margin repair (mostly the rule-forced timestamp steps, where the audio decides between
        # adjacent timestamps): lean the row towards one of the contenders if that raises the
        # smallest top-2 margin over the clips
        mm = min(_top2(x) for x in final)
        if mm < repair_margin:
            row = table[q].copy()
            cont = set()
            for x in final:
                cont.update(int(i) for i in np.argsort(-x)[:2])
            best = (mm, row)
            for u in sorted(cont):
                for beta in (1.0, 3.0, 8.0, -1.0, -3.0):
                    m2 = min(_top2(x) for x in evaluate(row + np.float32(beta) * E[u], q))
                    if m2 > best[0]:
                        best = (m2, row + np.float32(beta) * E[u])
            final = evaluate(best[1], q)
            n_repair += 1
            log(f"  q {q}: margin {mm:.4f} -> {best[0]:.4f}")
        am = [int(np.argmax(x)) for x in final]
        for (i, j) in pairs:
            if am[i] != am[j]:
                pairs[(i, j)] += 1
        assert st.eot not in am, f"<|endoftext|> at position {q}"
        for n, tok in zip(names, am):
            ids[n].append(tok)
            seq[n].append(tok)
            prev[n] = tok
        if q % 50 == 0:
            log(f"  q {q}: splits {n_split}, pair differences {dict((f'{names[i]}/{names[j]}', c) for (i, j), c in pairs.items())}")
    log(f"  splits {n_split}, margin repairs {n_repair}")
    return table.copy(), ids, n_split


def greedy_golden(model, d, enc, full_every: int | None, n_full_first: int = 4):
    """Greedy decoding of one window to <|endoftext|> or n_text_ctx positions with the
    openai / faster-whisper logits rules, on the fp32 transformers model: ids, the
    chosen log-probs, top-2 margins (after the rules), per-step lse and the logits of
    the step's top-32 + a fixed 256-token sample, and the full raw logits at the first
    n_full_first steps and every full_every-th step (None: first steps only)."""
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    suppress = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    gc = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                          max_initial_timestamp_index=50)

    def step(ids, past):
        with torch.no_grad():
            o = model(encoder_outputs=(enc,), decoder_input_ids=torch.tensor([ids]), past_key_values=past,
                      use_cache=True)
        return o.logits[0, -1].double(), o.past_key_values

    lg, past = step([st.sot], None)
    sot_logits = lg.float().numpy().copy()
    lang = st.first_lang + int(np.argmax(sot_logits[st.first_lang:st.first_lang + st.n_langs]))
    nsp = float(torch.softmax(lg, -1)[st.no_speech])
    prompt = [st.sot, lang, st.transcribe]
    lg, past = step([lang], past)
    lg, past = step([st.transcribe], past)
    begin = len(prompt)
    procs = [SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], begin),
             SuppressTokensLogitsProcessor(list(suppress)),
             WhisperTimeStampLogitsProcessor(gc, begin)]
    sample = np.sort(np.random.default_rng(2024).choice(d.n_vocab, TURBO_SUBSET, replace=False)).astype(np.int32)
    seq = list(prompt)
    ids, lps, full, full_steps, lse, sub_i, sub_v, margins = [], [], [], [], [], [], [], []
    sum_lp = 0.0
    while True:
        raw = lg.float().numpy()
        k = len(lse)
        if k < n_full_first or (full_every and k % full_every == 0):
            full.append(raw.copy())
            full_steps.append(k)
        lse.append(float(torch.logsumexp(lg, -1)))
        t32 = np.argsort(-raw, kind="stable")[:32].astype(np.int32)
        sub_i.append(np.concatenate([t32, sample]))
        sub_v.append(raw[sub_i[-1]])
        x = lg[None].clone().float()
        for p in procs:
            x = p(torch.tensor([seq]), x)
        lsm = torch.log_softmax(x.double(), -1)[0]
        top2 = torch.topk(x[0], 2).values
        margins.append(float(top2[0] - top2[1]))
        nxt = int(torch.argmax(x[0]))
        sum_lp += float(lsm[nxt])
        lps.append(float(lsm[nxt]))
        if nxt == st.eot:
            break
        ids.append(nxt)
        seq.append(nxt)
        if len(seq) >= d.n_text_ctx:
            break
        lg, past = step([nxt], past)
    return dict(sot_logits=sot_logits, full_logits=np.stack(full), full_steps=np.array(full_steps, np.int32),
                lse=np.array(lse), sub_ids=np.stack(sub_i), sub_vals=np.stack(sub_v), ids=np.array(ids, np.int32),
                logprobs=np.array(lps), margins=np.array(margins), language=np.int32(lang),
                no_speech_prob=np.float64(nsp), sum_logprob=np.float64(sum_lp))


def gen_turbo_text(out):
    """whisper-large-v3-turbo, text weights (TEXT_SEED, TEXT_AMP) with the audio-dependent
    positional table (construct_audio_table), three spectrally distinct 30 s clips: greedy
    to 448 positions each on the fp32 transformers model (full logits at the first 4 steps
    and every 32nd for the first clip, at the first 4 for the others), and beam 5 on the
    first clip.  The table is stored (pos_table): the GPU tests upload it."""
    from oracle import decode as odec

    d = D.LARGE_V3_TURBO
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=TEXT_SEED, text_pos=TEXT_AMP)
    model = build_model(d, w)
    encs = {}
    for name, make in TEXT_CLIPS.items():
        mel = fe_mel(make(), d.n_mels)[:, :3000]
        with torch.no_grad():
            encs[name] = model.model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
    table, cids, n_split = construct_audio_table(d, w, {n: e[0].numpy() for n, e in encs.items()})
    del w
    with torch.no_grad():
        model.model.decoder.embed_positions.weight.copy_(torch.from_numpy(table))
    store = {"pos_table": table.astype(np.float32)}
    meta = {"seed": TEXT_SEED, "text_pos": TEXT_AMP, "clips": list(TEXT_CLIPS), "per_clip": {},
            "construction": {"split_positions": n_split, "split_margin": TEXT_SPLIT_MARGIN,
                             "max_shift": TEXT_MAX_SHIFT}}
    for ci, name in enumerate(TEXT_CLIPS):
        enc = encs[name]
        g = greedy_golden(model, d, enc, TURBO_FULL_STRIDE if ci == 0 else None)
        assert g["ids"].tolist() == cids[name], f"{name}: transformers' ids differ from the construction's"
        e = enc[0].numpy()
        g["enc_rownorm"] = np.linalg.norm(e.astype(np.float64), axis=1)
        for k, v in g.items():
            store[f"{name}/{k}"] = v
        ids = g["ids"]
        meta["per_clip"][name] = {"n_ids": int(len(ids)), "distinct_ids": int(len(set(ids.tolist()))),
                                  "timestamp_ids": int((ids >= st.timestamp_begin).sum()),
                                  "min_top2_margin": float(g["margins"].min()),
                                  "p1_top2_margin": float(np.percentile(g["margins"], 1)),
                                  "logit_std": float(np.std(g["full_logits"][0]))}
        print("turbo text", name, meta["per_clip"][name], "first", ids[:10].tolist())
    names = list(TEXT_CLIPS)
    diffs = {}
    for i in range(len(names)):
        for j in range(i + 1, len(names)):
            x, y = store[names[i] + "/ids"], store[names[j] + "/ids"]
            n = min(len(x), len(y))
            diffs[f"{names[i]}/{names[j]}"] = int((x[:n] != y[:n]).sum() + abs(len(x) - len(y)))
    meta["pair_id_differences"] = diffs
    meta["min_top2_margin"] = min(v["min_top2_margin"] for v in meta["per_clip"].values())
    print("turbo text: pair differences", diffs, "min margin", meta["min_top2_margin"])
    assert min(diffs.values()) >= TEXT_MIN_PAIR_DIFF, diffs
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    r = odec.beam_from_encoder(_HFStepper(model, encs["chirp0"]), None, st,
                               opts=odec.DecodeOptions(suppress_tokens=sup, max_length=TURBO_BEAM_MAX_LEN),
                               beam=odec.BeamOptions(beam_size=5))
    store["beam5/ids"] = np.array(r.tokens, np.int32)
    store["beam5/sum_logprob"] = np.float64(r.sum_logprob)
    store["beam5/language"] = np.int32(r.language)
    store["beam5/no_speech_prob"] = np.float64(r.no_speech_prob)
    store["beam5/max_length"] = np.int32(TURBO_BEAM_MAX_LEN)
    meta["beam5"] = {"clip": "chirp0", "n_ids": len(r.tokens), "distinct_ids": len(set(r.tokens)),
                     "max_length": TURBO_BEAM_MAX_LEN}
    print("turbo text beam5", meta["beam5"], "first", r.tokens[:10])
    np.savez_compressed(os.path.join(out, "turbo_text.npz"), **store)
    return meta


# (Round 6 tried the constructed, audio-dependent table at tiny dims too: with the tiny text
# lean (TINY_TEXT_AMP 200, needed for the tiny GPU encoder's 1e-2 tolerance) no position had
# a cross-clip logit gap wide enough for a 0.3 split margin (0 splits), so the tiny golden
# keeps its one clip; the audio-dependence is pinned by the turbo golden.)
def gen_tiny_text(out):
    """tiny dims, text weights: greedy ids of one 30 s clip (the CPU oracle and the
    GPU are both held to them)."""
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=TEXT_SEED, text_pos=TINY_TEXT_AMP)
    model = build_model(d, w)
    mel = fe_mel(synth.chirp_clip(3, 30.0), d.n_mels)[:, :3000]
    with torch.no_grad():
        enc = model.model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
    g = greedy_golden(model, d, enc, None, n_full_first=8)
    g["mel"] = mel
    np.savez_compressed(os.path.join(out, "tiny_text.npz"), **g)
    ids = g["ids"]
    meta = {"seed": TEXT_SEED, "text_pos": TINY_TEXT_AMP, "clip": "chirp_clip(3, 30 s)", "n_ids": int(len(ids)),
            "distinct_ids": int(len(set(ids.tolist()))), "min_top2_margin": float(g["margins"].min())}
    print("tiny text", meta, "first", ids[:10].tolist())
    return meta


def gen_logits_rules(out):
    """Crafted token histories through transformers' Whisper processors."""
    st = D.SpecialTokens.for_vocab(51866)
    tok = WhisperTokenizer(51866)
    suppress = get_suppressed_tokens(tok, [-1])
    gc = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                          max_initial_timestamp_index=50)
    tb = st.timestamp_begin
    cases = [
        [],                                   # first step: timestamps only, <= 1.00 s
        [tb + 3],                             # after an opening timestamp
        [tb + 3, 400, 500],                   # text after timestamp
        [tb + 3, 400, tb + 40],               # closing timestamp -> pair rule
        [tb + 3, 400, tb + 40, tb + 40],      # two timestamps -> must be text
        [tb, 11, 12, tb + 7, tb + 7, 99],     # monotonic timestamps
        [1000, 2000, 3000],                   # no timestamps so far
        [tb + 1500],                          # last timestamp
    ]
    prompt = [st.sot, st.first_lang, st.transcribe]
    begin = len(prompt)
    procs = [SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], begin),
             SuppressTokensLogitsProcessor(list(suppress)),
             WhisperTimeStampLogitsProcessor(gc, begin)]
    masks, argmaxes, lens, flat = [], [], [], []
    for ci, hist in enumerate(cases):
        for variant in range(2):
            rng = np.random.default_rng(100 + 2 * ci + variant)
            lg = rng.standard_normal(51866).astype(np.float32) * 2.0
            if variant == 1:   # make timestamps likely to win the mass rule
                lg[tb:] += 4.0
            x = torch.from_numpy(lg)[None]
            seq = torch.tensor([prompt + hist])
            for p in procs:
                x = p(seq, x)
            masks.append(np.packbits(~torch.isfinite(x[0]).numpy()))
            argmaxes.append(int(torch.argmax(x[0])))
            lens.append(len(hist))
            flat.extend(hist)
    np.savez_compressed(os.path.join(out, "logits_rules.npz"), masks=np.stack(masks),
                        argmax=np.array(argmaxes, np.int32), hist_len=np.array(lens, np.int32),
                        hist=np.array(flat, np.int32), suppress=np.array(suppress, np.int32))
    return {"n_cases": len(masks)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    ap.add_argument("--only", default=None,
                    help="comma list of: mel,rules,tiny,turbo_layer,turbo,turbo_beam,tiny_text,turbo_text")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    torch.manual_seed(0)
    mp = os.path.join(a.out, "meta.json")
    meta = json.load(open(mp)) if os.path.exists(mp) else {}
    meta.update({"generator": "tools/make_golden.py", "transformers": __import__("transformers").__version__,
                 "torch": torch.__version__})
    only = set(a.only.split(",")) if a.only else {"mel", "rules", "tiny", "turbo_layer", "turbo", "turbo_beam",
                                                 "tiny_text", "turbo_text"}
    if "mel" in only:
        meta["mel"] = gen_mel(a.out)
    if "rules" in only:
        meta["logits_rules"] = gen_logits_rules(a.out)
    if "tiny" in only:
        meta["tiny"] = gen_tiny(a.out)
    if "turbo_layer" in only:
        meta["turbo_layer"] = gen_turbo_layer(a.out)
    if "turbo" in only:
        meta["turbo"] = gen_turbo(a.out)
    if "turbo_beam" in only:
        meta["turbo_beam"] = gen_turbo_beam(a.out)
    if "tiny_text" in only:
        meta["tiny_text"] = gen_tiny_text(a.out)
    if "turbo_text" in only:
        meta["turbo_text"] = gen_turbo_text(a.out)
    with open(os.path.join(a.out, "meta.json"), "w") as fh:
        json.dump(meta, fh, indent=1)


if __name__ == "__main__":
    main()
