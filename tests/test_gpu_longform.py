"""Long-form transcription (> 30 s, faster-whisper's seek loop with
condition_on_previous_text) through the backend's batched seek loop
(open-speech_amd/segments.py:transcribe_clips) on the GPU, checked window by window
against the oracle's restatement of generate_segments (oracle/seek.py): the same
window positions and sizes, the same previous-text prompts, token ids identical to the
fp16-emulating oracle decoding the GPU's own encoder output of each window, and the
same segments.  Greedy (beam_size=1, the parity mode)."""
import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth, weights
from open_speech_amd.engine import WhisperEngine
from open_speech_amd.segments import TranscribeOptions, transcribe_clips
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

pytestmark = pytest.mark.gpu


class Recorder:
    """The engine seam of transcribe_clips, recording each encoded window's encoder
    output and each decode call's prompts and outputs."""

    def __init__(self, eng):
        self.eng, self.max_batch, self.max_rows = eng, eng.max_batch, eng.max_rows
        self.enc, self.calls, self._wins = {}, [], []

    def log_mel(self, clips):
        return self.eng.log_mel(clips)

    def encode(self, wins):
        self._wins = list(wins)
        self.eng.encode(wins)
        for k, (_clip, seek, size) in enumerate(wins):
            self.enc[(seek, size)] = self.eng.encoder_output(k)

    def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
        outs = self.eng.decode(n, cfg, prefix=prefix, languages=languages)
        for k, w in enumerate(self._wins):
            self.calls.append((w[1], w[2], list(prefix[k]) if prefix else [], outs[k]))
        return outs


def test_longform_seek_loop_matches_oracle():
    from oracle import decode as odec
    from oracle import seek as oseek
    from oracle.model import WhisperOracle
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=1234, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=2)
    try:
        eng.load_weights(w)
        tok = WhisperTokenizer(d.n_vocab)
        st = tok.special
        sup = get_suppressed_tokens(tok, [-1])
        pcm = synth.chirp_clip(41, 75.0)
        rec = Recorder(eng)
        res = transcribe_clips(rec, [pcm], TranscribeOptions(beam_size=1), tok, sup)[0]
        gpu = {(s, z): (p, o) for s, z, p, o in rec.calls}
        assert len(rec.calls) >= 3, "a 75 s clip needs at least three 30 s windows"

        orc = WhisperOracle(d, w, fp16=True)
        lang = {}

        def decode_window(seek, size, prompt):
            assert (seek, size) in rec.enc, f"the GPU never encoded window (seek {seek}, size {size})"
            enc = rec.enc[(seek, size)]
            r = odec.greedy_from_encoder(orc, orc.cross_kv(enc), st, language=lang.get("tok"),
                                         prev_tokens=prompt[1:], opts=odec.DecodeOptions(suppress_tokens=sup))
            lang.setdefault("tok", r.language)
            gp, go = gpu[(seek, size)]
            assert gp == prompt, f"window {seek}: prompt differs"
            assert go.tokens == r.tokens, f"window {seek}: GPU ids differ from the oracle's"
            assert abs(go.no_speech_prob - r.no_speech_prob) < 2e-3
            return go.tokens, go.sum_logprob, go.no_speech_prob

        nf = (len(pcm) + 160) // 160
        wins = oseek.seek_loop(decode_window, nf, st, tok.decode)
        assert [(x.seek, x.size) for x in wins] == [(s, z) for s, z, _, _ in rec.calls]
        want = [(a, b, t) for x in wins for a, b, t in x.segments]
        got = [(sg.start, sg.end, sg.tokens) for sg in res.segments]
        assert got == want
        assert res.duration == pytest.approx(75.0)
    finally:
        eng.close()


def test_longform_beam5_seek_loop_matches_oracle():
    """The reference's decoding (beam_size 5, src/backends/faster_whisper.py:237) inside
    the seek loop: a 75 s clip through transcribe_clips with beam 5, every window's
    prompt and ids equal to the oracle's CTranslate2-BeamSearch restatement decoding the
    GPU's own encoder output, and the same segments.  faster-whisper's max_new_tokens
    (24 per window) bounds the oracle's cost: random weights never emit <|endoftext|>."""
    from oracle import decode as odec
    from oracle import seek as oseek
    from oracle.model import WhisperOracle
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=1234, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=2)
    try:
        eng.load_weights(w)
        tok = WhisperTokenizer(d.n_vocab)
        st = tok.special
        sup = get_suppressed_tokens(tok, [-1])
        pcm = synth.chirp_clip(42, 75.0)
        rec = Recorder(eng)
        opts = TranscribeOptions(beam_size=5, max_new_tokens=24)
        res = transcribe_clips(rec, [pcm], opts, tok, sup)[0]
        gpu = {(s, z): (p, o) for s, z, p, o in rec.calls}
        assert len(rec.calls) >= 3
        orc = WhisperOracle(d, w, fp16=True)
        lang = {}

        def decode_window(seek, size, prompt):
            enc = rec.enc[(seek, size)]
            plen = len(prompt) + 3
            r = odec.beam_from_encoder(orc, orc.cross_kv(enc), st, language=lang.get("tok"), prev_tokens=prompt[1:],
                                       opts=odec.DecodeOptions(suppress_tokens=sup, max_length=plen + 24),
                                       beam=odec.BeamOptions(beam_size=5))
            lang.setdefault("tok", r.language)
            gp, go = gpu[(seek, size)]
            assert gp == prompt, f"window {seek}: prompt differs"
            assert go.tokens == r.tokens, f"window {seek}: GPU beam ids differ from the oracle's"
            assert abs(go.sum_logprob - r.sum_logprob) <= 1e-4 * (len(r.tokens) + 1) + 1e-3 * abs(r.sum_logprob)
            return go.tokens, go.sum_logprob, go.no_speech_prob

        nf = (len(pcm) + 160) // 160
        wins = oseek.seek_loop(decode_window, nf, st, tok.decode)
        assert [(x.seek, x.size) for x in wins] == [(s, z) for s, z, _, _ in rec.calls]
        want = [(a, b, t) for x in wins for a, b, t in x.segments]
        assert [(sg.start, sg.end, sg.tokens) for sg in res.segments] == want
    finally:
        eng.close()
