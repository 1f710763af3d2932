"""Row refill (osw_transcribe_refill, osw.hip decode_refill): more clips than decoder rows,
every row on its own step counter, a finished window's row refilled with the next queued
clip's window (encoded straight into that row's cross-K/V slot).  Rows are independent in
every kernel, so each clip must decode exactly as in a plain osw_transcribe_batch call:
same ids, bit-equal sum_logprob and no-speech probability, same language."""
import dataclasses

import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth, weights
from open_speech_amd.engine import DecodeConfig, WhisperEngine
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

pytestmark = pytest.mark.gpu


def _check(eng, clips, cfg, budgets, refill_min, chunk):
    got = eng.transcribe_refill(clips, dataclasses.replace(cfg, token_budget=tuple(budgets)), refill_min=refill_min)
    assert len(got) == len(clips)
    for i0 in range(0, len(clips), chunk):
        ref = eng.transcribe_batch(clips[i0:i0 + chunk],
                                   dataclasses.replace(cfg, token_budget=tuple(budgets[i0:i0 + chunk])))
        for j, r in enumerate(ref):
            g = got[i0 + j]
            assert g.tokens == r.tokens, i0 + j
            assert g.sum_logprob == r.sum_logprob, i0 + j
            assert g.no_speech_prob == r.no_speech_prob, i0 + j
            assert g.language == r.language, i0 + j
    return got


@pytest.mark.parametrize("refill_min", [1, 3, 8])
def test_refill_matches_batch_tiny(refill_min):
    """21 clips (30 s and 12.5 s) through 8 rows, budgets 5..27 tokens so rows finish at
    different steps and every row is refilled several times."""
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=1234, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=8)
    try:
        eng.load_weights(w)
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=64)
        clips = [synth.chirp_clip(30 + i, 30.0 if i % 3 else 12.5) for i in range(21)]
        budgets = [5 + (7 * i) % 23 for i in range(21)]
        got = _check(eng, clips, cfg, budgets, refill_min, 7)
        assert len({len(g.tokens) for g in got}) > 3  # the windows really end at different steps
    finally:
        eng.close()


def test_refill_fewer_clips_than_rows_and_no_budget():
    """5 clips in 8 rows, no token budget (max_length ends them): no refill happens, only
    the per-row step counters differ from the plain path."""
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=99, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=8)
    try:
        eng.load_weights(w)
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=40)
        clips = [synth.chirp_clip(70 + i, 30.0) for i in range(5)]
        got = eng.transcribe_refill(clips, cfg, refill_min=4)
        ref = eng.transcribe_batch(clips, cfg)
        for g, r in zip(got, ref):
            assert g.tokens == r.tokens and g.sum_logprob == r.sum_logprob and g.language == r.language
    finally:
        eng.close()


def test_refill_matches_batch_turbo():
    """large-v3-turbo dims (random weights): 12 clips through 8 rows."""
    d = D.LARGE_V3_TURBO
    eng = WhisperEngine(d, device=0, max_batch=8)
    try:
        eng.init_random(seed=3)
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=40)
        clips = [synth.chirp_clip(90 + i, 30.0) for i in range(12)]
        budgets = [3 + (5 * i) % 17 for i in range(12)]
        _check(eng, clips, cfg, budgets, 2, 6)
    finally:
        eng.close()


def test_refill_rejects_beam_search():
    d = D.MICRO_TEST
    eng = WhisperEngine(d, device=0, max_batch=4)
    try:
        eng.load_weights(weights.random_weights(d, seed=1, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        with pytest.raises(Exception, match="greedily"):
            eng.transcribe_refill([synth.chirp_clip(1, 5.0)], DecodeConfig(suppress_tokens=sup, beam_size=5,
                                                                           max_length=16))
    finally:
        eng.close()
