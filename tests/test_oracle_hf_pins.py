"""The oracle's beam-search restatement pinned against transformers' own beam search
(an independent implementation; tools/make_hf_pins.py, tests/golden/hf_beam_pins.npz).

The fixtures hold what transformers 5.15.0 ``GenerationMixin._beam_search`` returned
(width 5, early_stopping=True, 5 returned sequences) on tiny-test dims, in the three
configurations where its semantics and CTranslate2's (as the oracle restates it)
coincide: no logits processor (``plain``); Whisper's processors with the log-softmax
renormalisation CT2 applies (``rules``); and length penalty 1 with the oracle's
``length_counts_eot`` set to transformers' length convention (``lp1``).  Each case is
replayed here by the oracle's own numpy model (fp32) on the same encoder output: the
best hypothesis and the five best finished hypotheses must be identical, the scores
within 1e-3.  CT2's defaults that transformers lacks (num_hypotheses = 1 with its
"top candidate finished" stop, the length without <|endoftext|>) stay unpinned
(DESIGN.md §2)."""
import json
import os

import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import weights
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens
from oracle import decode as odec
from oracle.model import WhisperOracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLD, "meta.json")))["hf_beam_pins"]
CASES = {"plain": (False, 0.0, "plain"), "rules": (True, 0.0, "rules"), "lp1": (True, 1.0, "rules")}


def _weights(d, mix):
    w = weights.random_weights(d, seed=META["seed"], emb_std=META["emb_std"])
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    tok = w["dec.tok"].astype(np.float32)
    tok[st.eot] = sum(f * tok[t] for t, f in mix)
    w["dec.tok"] = tok.astype(w["dec.tok"].dtype)
    return w


@pytest.fixture(scope="module")
def pins():
    d = D.TINY_TEST
    z = np.load(os.path.join(GOLD, "hf_beam_pins.npz"))
    orcs = {k: WhisperOracle(d, _weights(d, m), fp16=False) for k, m in META["eot_mix"].items()}
    return d, z, orcs


@pytest.mark.parametrize("ci", [0])
@pytest.mark.parametrize("name", list(CASES))
def test_oracle_beam_equals_transformers(pins, name, ci):
    d, z, orcs = pins
    rules, lp, mk = CASES[name]
    key = f"{name}_{ci}"
    assert META["cases"][key]["length_penalty"] == lp and META["cases"][key]["rules"] == rules
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    orc = orcs[mk]
    xkv = orc.cross_kv(z[f"enc{ci}"])
    opts = odec.DecodeOptions(suppress_blank=rules, suppress_tokens=sup if rules else (),
                              without_timestamps=not rules, max_length=META["max_length"])
    bo = odec.BeamOptions(beam_size=META["beam"], num_hypotheses=META["beam"], length_penalty=lp,
                          length_counts_eot=lp != 0)
    r = odec.beam_from_encoder(orc, xkv, st, language=st.first_lang, opts=opts, beam=bo)
    lens = z[key + "_lens"].tolist()
    flat = z[key + "_ids"].tolist()
    hf, off = [], 0
    for n in lens:
        hf.append(flat[off:off + n])
        off += n
    scores = z[key + "_scores"]
    assert r.tokens == hf[0]
    # transformers keeps the best `beam` finished hypotheses by normalised score
    mine = sorted(r.hypotheses, key=lambda h: -h[2])[:len(hf)]
    assert [h[0] for h in mine] == hf
    np.testing.assert_allclose([h[2] for h in mine], scores, atol=1e-3, rtol=0)
