"""The oracle's long-form seek loop (oracle/seek.py, faster-whisper's generate_segments
restated) pinned against transformers' own long-form sequential generation on a 75 s
clip (tools/make_hf_longform_pin.py, tests/golden/hf_longform_pin.npz): temperature 0,
condition on previous text, no-speech and log-prob thresholds on, timestamps on.

The fixture is transformers' segment list; here the oracle's seek loop with the oracle's
own numpy model (fp32) and the same position-scheduled logit bias
(tests/hf_longform_pin.py) must reproduce every segment: tokens, start and end.  The
generator checked the same equality with transformers' decoder driving the oracle."""
import json
import os

import numpy as np

from hf_longform_pin import bias_row
from open_speech_amd import dims as D
from open_speech_amd import synth, weights
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens
from oracle import decode as odec
from oracle import mel as omel
from oracle import seek as oseek
from oracle.model import WhisperOracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
META = json.load(open(os.path.join(GOLD, "meta.json")))["hf_longform_pin"]


class _Biased:
    """WhisperOracle's decoder-step interface with the pin's logit bias added."""

    def __init__(self, orc, st, n_vocab):
        self.orc, self.st, self.V = orc, st, n_vocab

    def new_cache(self):
        return self.orc.new_cache()

    def decoder_step(self, tok, pos, cache, xkv):
        return self.orc.decoder_step(tok, pos, cache, xkv) + bias_row(pos, self.st, self.V)


def test_oracle_seek_loop_equals_transformers_longform():
    d = D.TINY_TEST
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    w = weights.random_weights(d, seed=META["seed"], emb_std=META["emb_std"])
    orc = WhisperOracle(d, w, fp16=False)
    biased = _Biased(orc, st, d.n_vocab)
    mel = omel.log_mel(omel.pcm16_to_float(synth.chirp_clip(META["clip"], META["seconds"])), d.n_mels)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    opts = odec.DecodeOptions(suppress_tokens=sup)

    def decode_window(seek, size, prompt):
        x = np.zeros((d.n_mels, 3000), np.float32)
        x[:, :size] = mel[:, seek:seek + size]
        xkv = orc.cross_kv(orc.encode(x))
        r = odec.greedy_from_encoder(biased, xkv, st, language=st.first_lang,
                                     prev_tokens=prompt[1:] if prompt else (), opts=opts)
        return r.tokens, r.sum_logprob, r.no_speech_prob

    wins = oseek.seek_loop(decode_window, mel.shape[1], st, lambda t: "x")
    assert [[x.seek, x.size, len(x.prompt), len(x.tokens), x.skipped] for x in wins] == META["windows"]
    z = np.load(os.path.join(GOLD, "hf_longform_pin.npz"))
    segs = [(a, b, t) for x in wins for a, b, t in x.segments]
    lens = z["lens"].tolist()
    assert [len(t) for _, _, t in segs] == lens
    flat = z["ids"].tolist()
    off = 0
    for (a, b, t), a1, b1, n in zip(segs, z["starts"], z["ends"], lens):
        assert t == flat[off:off + n]
        off += n
        assert abs(a - a1) < 1e-6 and abs(b - b1) < 1e-6
