#!/usr/bin/env python3
"""Pin the oracle's beam-search restatement against transformers' own beam search
(run here, on CPU; writes tests/golden/hf_beam_pins.npz + a meta entry; committed).

The oracle's ``beam_from_encoder`` (oracle/decode.py) restates CTranslate2's
``BeamSearch`` [upstream, not installed].  Its golden (``turbo_beam5.npz``) was made by
that same restatement, so round 3 checked it only against itself.
Here an independent implementation -- transformers 5.15.0 ``GenerationMixin._beam_search``
(generation/utils.py:3208-3530) -- decodes the same encoder output, in configurations
where the two algorithms' semantics coincide:

* ``num_hypotheses = beam_size`` and ``patience = 1``: CT2 stops once 5 hypotheses are
  finished (round(beam*patience)), as transformers does with ``early_stopping=True``
  (``_beam_search_has_unfinished_sequences``, :3055-3075); CT2's "top candidate
  finished and >= num_hypotheses" rule cannot fire earlier.
* finished candidates come from the first ``beam`` ranks only (CT2 and transformers'
  ``top_num_beam_mask``); the surviving beams are the ``beam`` best unfinished of the
  ``2*beam`` candidates in both (CT2 refills slots in rank order, transformers re-sorts:
  the same set).
* logits rules: transformers applies its processors to log-probabilities without
  renormalising (:3388-3389); CT2 processes the logits and then takes the log-softmax.
  Case ``rules`` appends a log-softmax processor after transformers' Whisper processors
  (SuppressTokensAtBegin, SuppressTokens, WhisperTimeStamp) so both score the same
  renormalised distribution; case ``plain`` has no processor at all (nothing to
  renormalise).
* length normalisation: transformers divides by the generated length INCLUDING the
  <|endoftext|> (:3182); the CT2 restatement by the token count without it.  Cases with
  ``length_penalty = 0`` need no normalisation; case ``lp1`` sets the oracle's
  ``length_counts_eot`` to transformers' convention.

Each case is decoded twice here: by transformers' beam search and by the oracle's
restatement driven by transformers' decoder (``make_golden._HFStepper``, so both see
identical logits); the generator asserts they agree, then stores transformers' result.
``tests/test_oracle_hf_pins.py`` replays every case with the oracle's own numpy model
(fp32) on the stored encoder output.

The model is tiny-test (d 384) with hash weights at ``emb_std`` 0.1 and the
<|endoftext|> embedding row set to a mix of the rows of tokens 2452 and 38915 (``EOT_MIX``:
the tokens these random weights collapse to without and with the timestamp rules), so
<|endoftext|> ranks among the candidates and hypotheses finish at different steps (with
plain random weights none ever finishes before max_length).

Usage:  python tools/make_hf_pins.py [--out tests/golden]
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
import make_golden as mg  # noqa: E402

from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth, weights  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402
from oracle import decode as odec  # noqa: E402

from transformers import GenerationConfig  # noqa: E402
from transformers.generation.logits_process import LogitsProcessor, LogitsProcessorList  # noqa: E402
from transformers.generation.utils import GenerationMixin  # noqa: E402
from transformers.modeling_outputs import BaseModelOutput  # noqa: E402

SEED = 1234
EMB_STD = 0.1
# <|endoftext|> row per case: the plain decode collapses to token 2452, the one under the
# timestamp rules to 38915
EOT_MIX = {"plain": ((2452, 0.7), (38915, 0.3)), "rules": ((38915, 0.9), (2452, 0.1))}
CLIPS = (3,)
MAX_LEN = 60
BEAM = 5


def pin_weights(d, mix):
    w = weights.random_weights(d, seed=SEED, emb_std=EMB_STD)
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    tok = w["dec.tok"].astype(np.float32)
    tok[st.eot] = sum(f * tok[t] for t, f in mix)
    w["dec.tok"] = tok.astype(w["dec.tok"].dtype)
    return w


class _Renorm(LogitsProcessor):
    """log_softmax over what the Whisper processors kept: CT2's processed log-probs."""

    def __call__(self, input_ids, scores):
        return torch.log_softmax(scores, dim=-1)


CASES = {
    # name: (timestamp / suppression rules on, length_penalty, EOT_MIX key)
    "plain": (False, 0.0, "plain"),
    "rules": (True, 0.0, "rules"),
    "lp1": (True, 1.0, "rules"),
}


def hf_beam(model, enc, st, rules: bool, lp: float, sup):
    prompt = [st.sot, st.first_lang, st.transcribe] + ([] if rules else [st.no_timestamps])
    procs = LogitsProcessorList()
    if rules:
        gcfg = GenerationConfig(no_timestamps_token_id=st.no_timestamps, eos_token_id=st.eot,
                                max_initial_timestamp_index=50)
        begin = len(prompt)
        procs.extend([mg.SuppressTokensAtBeginLogitsProcessor([st.blank, st.eot], begin),
                      mg.SuppressTokensLogitsProcessor(list(sup)),
                      mg.WhisperTimeStampLogitsProcessor(gcfg, begin), _Renorm()])
    gc = GenerationConfig(num_beams=BEAM, early_stopping=True, length_penalty=lp, max_length=MAX_LEN,
                          eos_token_id=st.eot, pad_token_id=st.eot, decoder_start_token_id=st.sot, do_sample=False,
                          num_return_sequences=BEAM, output_scores=True, return_dict_in_generate=True)
    out = GenerationMixin.generate(model, decoder_input_ids=torch.tensor([prompt]),
                                   encoder_outputs=BaseModelOutput(last_hidden_state=enc), generation_config=gc,
                                   logits_processor=procs)
    hyps = []
    for seq, sc in zip(out.sequences.tolist(), out.sequences_scores.tolist()):
        gen = seq[len(prompt):]
        toks = gen[:gen.index(st.eot)] if st.eot in gen else gen
        hyps.append((toks, float(sc)))
    return hyps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden"))
    a = ap.parse_args()
    torch.manual_seed(0)
    d = D.TINY_TEST
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    models = {k: mg.build_model(d, pin_weights(d, m)) for k, m in EOT_MIX.items()}
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    store, meta = {}, {"generator": "tools/make_hf_pins.py", "seed": SEED, "emb_std": EMB_STD, "eot_mix": EOT_MIX,
                       "max_length": MAX_LEN, "beam": BEAM, "cases": {}}
    for ci, clip in enumerate(CLIPS):
        pcm = synth.chirp_clip(clip, 30.0)
        mel = mg.fe_mel(pcm, d.n_mels)[:, :3000]
        # the encoder does not read dec.tok: one encoder output serves both weight sets
        with torch.no_grad():
            enc = models["plain"].model.encoder(input_features=torch.from_numpy(mel)[None]).last_hidden_state
        store[f"enc{ci}"] = enc[0].numpy().astype(np.float32)
        for name, (rules, lp, mk) in CASES.items():
            model = models[mk]
            hyps = hf_beam(model, enc, st, rules, lp, sup)
            opts = odec.DecodeOptions(suppress_blank=rules, suppress_tokens=sup if rules else (),
                                      without_timestamps=not rules, max_length=MAX_LEN)
            bo = odec.BeamOptions(beam_size=BEAM, num_hypotheses=BEAM, length_penalty=lp, length_counts_eot=lp != 0)
            r = odec.beam_from_encoder(mg._HFStepper(model, enc), None, st, language=st.first_lang, opts=opts,
                                       beam=bo)
            assert r.tokens == hyps[0][0], (name, clip, r.tokens, hyps[0][0])
            n_fin = [len(t) for t, _ in hyps]
            key = f"{name}_{ci}"
            flat = [t for toks, _ in hyps for t in toks]
            store[key + "_ids"] = np.array(flat, np.int32)
            store[key + "_lens"] = np.array(n_fin, np.int32)
            store[key + "_scores"] = np.array([s for _, s in hyps], np.float64)
            meta["cases"][key] = {"clip": clip, "rules": rules, "length_penalty": lp, "best_len": len(hyps[0][0]),
                                  "hyp_lens": n_fin, "oracle_finished": len(r.hypotheses)}
            print(key, "best", hyps[0][0][:12], "lens", n_fin, "scores", [round(s, 4) for _, s in hyps],
                  "oracle finished", len(r.hypotheses))
    np.savez_compressed(os.path.join(a.out, "hf_beam_pins.npz"), **store)
    mp = os.path.join(a.out, "meta.json")
    m = json.load(open(mp)) if os.path.exists(mp) else {}
    m["hf_beam_pins"] = meta
    with open(mp, "w") as fh:
        json.dump(m, fh, indent=1)


if __name__ == "__main__":
    main()
