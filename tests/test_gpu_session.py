"""Decode sessions (osw_session_*, osw.hip session_step): windows of different clips, seeks,
prefixes and languages admitted into free decoder slots between chunks of decoder steps,
each slot's rows on their own step counter.  Every row's arithmetic is the plain decode's
(rows are independent in every kernel), so each window must decode exactly as it does
alone through osw_encode_windows + osw_decode_windows: same ids, bit-equal sum_logprob and
no-speech probability, same language — greedy and beam search."""
import dataclasses

import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth, weights
from open_speech_amd.dims import SpecialTokens
from open_speech_amd.engine import DecodeConfig, WhisperEngine
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

pytestmark = pytest.mark.gpu


def _windows(d, n, seed0):
    st = SpecialTokens.for_vocab(d.n_vocab)
    out = []
    for i in range(n):
        secs = (30.0, 12.5, 47.0)[i % 3]
        pcm = synth.chirp_clip(seed0 + i, secs)
        nf = len(pcm) // 160 + 1
        seek = (0, 700, 1500)[i % 3] if secs > 40 else 0
        size = min(3000, nf - 1 - seek)
        prefix = None
        if i % 4 == 1:
            prefix = [st.sot_prev] + [100 + (13 * i + 7 * j) % 300 for j in range(3 + i % 5)]
        lang = None if i % 2 else st.first_lang + (i % 7)
        out.append(dict(tag=1000 + i, pcm=pcm, seek=seek, segment_size=size, language_token=lang, prefix=prefix,
                        token_budget=4 + (7 * i) % 19))
    return out


def _alone(eng, w, cfg):
    """The window decoded on its own, twice in one call: a batch-1 greedy decode would pick
    its tokens in the logits GEMM's epilogue (SelFuse), whose no-speech softmax sums in
    another order than the select kernel every multi-row decode uses."""
    eng.log_mel([w["pcm"]])
    eng.encode([(0, w["seek"], w["segment_size"])] * 2)
    c = dataclasses.replace(cfg, token_budget=(w["token_budget"],) * 2)
    return eng.decode(2, c, prefix=[w["prefix"]] * 2 if w["prefix"] else None, languages=[w["language_token"]] * 2)[0]


def _run_session(eng, cfg, wins, add_in=(1.0,), refill_min=1):
    """Add the windows in portions (fractions of the list) between steps; collect results."""
    eng.session_begin(cfg)
    got = {}
    try:
        cut = [0] + [int(round(f * len(wins))) for f in add_in]
        parts = [wins[a:b] for a, b in zip(cut, cut[1:])]
        eng.session_add(parts[0])
        k = 1
        guard = 0
        while True:
            res, active, queued = eng.session_step(max_chunks=2, refill_min=refill_min)
            for tag, out in res:
                assert tag not in got
                got[tag] = out
            if k < len(parts):
                eng.session_add(parts[k])
                k += 1
                continue
            if active == 0 and queued == 0:
                break
            guard += 1
            assert guard < 2000
    finally:
        eng.session_end()
    assert sorted(got) == sorted(w["tag"] for w in wins)
    return got


def _compare(eng, cfg, wins, got):
    for w in wins:
        r = _alone(eng, w, cfg)
        g = got[w["tag"]]
        assert g.tokens == r.tokens, w["tag"]
        assert g.sum_logprob == r.sum_logprob, w["tag"]
        assert g.no_speech_prob == r.no_speech_prob, w["tag"]
        assert g.language == r.language, w["tag"]


@pytest.mark.parametrize("beam", [1, 5])
def test_session_matches_alone_tiny(beam):
    """17 windows (3 clip lengths, seeks into a 47 s clip, prefixes, detected and fixed
    languages, budgets 4..22 tokens) through 6 slots, added in three portions while
    earlier ones decode."""
    d = D.TINY_TEST
    eng = WhisperEngine(d, device=0, max_batch=6)
    try:
        eng.load_weights(weights.random_weights(d, seed=4321, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=64, beam_size=beam)
        wins = _windows(d, 17, 200)
        got = _run_session(eng, cfg, wins, add_in=(0.3, 0.6, 1.0))
        _compare(eng, cfg, wins, got)
        assert len({len(g.tokens) for g in got.values()}) > 3
    finally:
        eng.close()


def test_session_no_budget_without_timestamps():
    """max_length ends the windows; <|notimestamps|> prompts; refill only when 3 slots are free."""
    d = D.TINY_TEST
    eng = WhisperEngine(d, device=0, max_batch=4)
    try:
        eng.load_weights(weights.random_weights(d, seed=77, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=40, without_timestamps=True)
        wins = _windows(d, 9, 300)
        for w in wins:
            w["token_budget"] = 0
        got = _run_session(eng, cfg, wins, refill_min=3)
        _compare(eng, cfg, wins, got)
    finally:
        eng.close()


@pytest.mark.parametrize("beam", [1, 5])
def test_session_matches_alone_turbo(beam):
    """large-v3-turbo dims (random weights): 10 windows through 4 slots."""
    d = D.LARGE_V3_TURBO
    eng = WhisperEngine(d, device=0, max_batch=4)
    try:
        eng.init_random(seed=5)
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=48, beam_size=beam)
        wins = _windows(d, 10, 400)
        got = _run_session(eng, cfg, wins, add_in=(0.5, 1.0))
        _compare(eng, cfg, wins, got)
    finally:
        eng.close()


def test_session_rejects_other_calls_and_sampling():
    d = D.MICRO_TEST
    eng = WhisperEngine(d, device=0, max_batch=4)
    try:
        eng.load_weights(weights.random_weights(d, seed=1, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        with pytest.raises(Exception, match="temperature 0"):
            eng.session_begin(DecodeConfig(suppress_tokens=sup, temperature=0.5, max_length=16))
        eng.session_begin(DecodeConfig(suppress_tokens=sup, max_length=16))
        with pytest.raises(Exception, match="session is open"):
            eng.transcribe_batch([synth.chirp_clip(1, 5.0)], DecodeConfig(suppress_tokens=sup, max_length=16))
        with pytest.raises(Exception, match="seek out of range"):
            eng.session_add([dict(tag=1, pcm=synth.chirp_clip(1, 5.0), seek=600, segment_size=10)])
        eng.session_end()
        out = eng.transcribe_batch([synth.chirp_clip(1, 5.0)], DecodeConfig(suppress_tokens=sup, max_length=16))
        assert len(out) == 1
    finally:
        eng.close()


def test_session_end_midway_then_new_session():
    """A session ended with windows still decoding and queued leaves the context usable: a
    new session (another decode configuration) and a plain batch decode give the same
    results as on a fresh context."""
    d = D.TINY_TEST
    eng = WhisperEngine(d, device=0, max_batch=4)
    try:
        eng.load_weights(weights.random_weights(d, seed=4321, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        wins = _windows(d, 9, 500)
        eng.session_begin(DecodeConfig(suppress_tokens=sup, max_length=64, beam_size=5))
        eng.session_add(wins)
        eng.session_step(max_chunks=1)
        eng.session_end()                     # 4 decoding, 5 queued: dropped
        cfg = DecodeConfig(suppress_tokens=sup, max_length=64)
        got = _run_session(eng, cfg, wins[:6])
        _compare(eng, cfg, wins[:6], got)
    finally:
        eng.close()


def test_session_clip_keys_match_own_pcm():
    """Resident clip log-mels (osw_session_window::clip): the windows of a 95 s
    clip and a 47 s clip queued by key — PCM with each clip's first window only, later
    windows staged from the clip's log-mel kept on the device — decode exactly as the same
    windows queued with their own PCM, and as each window alone.  A released key needs its
    PCM again."""
    d = D.TINY_TEST
    st = SpecialTokens.for_vocab(d.n_vocab)
    eng = WhisperEngine(d, device=0, max_batch=3)
    try:
        eng.load_weights(weights.random_weights(d, seed=99, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=48, beam_size=1)
        long_, mid = synth.chirp_clip(901, 95.0), synth.chirp_clip(902, 47.0)
        wins = []
        for key, pcm, seeks in ((7, long_, (0, 2900, 5600, 8100, 9300)), (8, mid, (0, 1800, 4000))):
            nf = len(pcm) // 160 + 1
            for j, sk in enumerate(seeks):
                wins.append(dict(tag=100 * key + j, clip=key, pcm=pcm if j == 0 else None, seek=sk,
                                 segment_size=min(3000, nf - 1 - sk), language_token=st.first_lang,
                                 prefix=[st.sot_prev, 300 + j] if j else None, token_budget=6 + 3 * j))
        own = [dict(w, clip=None, pcm=long_ if w["tag"] < 800 else mid) for w in wins]
        got_key = _run_session(eng, cfg, wins, add_in=(0.4, 0.7, 1.0))
        got_own = _run_session(eng, cfg, own, add_in=(0.4, 0.7, 1.0))
        for w in wins:
            a, b = got_key[w["tag"]], got_own[w["tag"]]
            assert (a.tokens, a.sum_logprob, a.no_speech_prob, a.language) == \
                (b.tokens, b.sum_logprob, b.no_speech_prob, b.language), w["tag"]
        _compare(eng, cfg, own, got_key)
        # a key is forgotten after release (and after session_end): its windows need PCM again
        eng.session_begin(cfg)
        try:
            eng.session_add([wins[0], dict(wins[1])])
            with pytest.raises(Exception, match="queued window"):
                eng.session_release_clip(7)             # a queued window still reads it
            eng.session_step(max_chunks=0)              # both admitted (staged from the clip)
            eng.session_release_clip(7)
            with pytest.raises(Exception, match="seek out of range"):
                eng.session_add([dict(wins[2])])        # key 7 is gone and this window has no PCM
        finally:
            eng.session_end()
    finally:
        eng.close()


def test_session_long_clip_admission_does_not_grow():
    """The per-window admission cost of a 20-minute clip's later windows (staged from its
    resident log-mel) is not the whole-clip upload + log-mel it was: it stays
    within a small factor of a 30 s clip's (timings printed with -s)."""
    import time

    import numpy as np
    d = D.TINY_TEST
    st = SpecialTokens.for_vocab(d.n_vocab)
    eng = WhisperEngine(d, device=0, max_batch=2)
    try:
        eng.load_weights(weights.random_weights(d, seed=5, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=24)
        eng.session_begin(cfg)
        try:
            def admit(key, pcm, seek, first):
                t = time.perf_counter()
                eng.session_add([dict(tag=key * 1000 + seek, clip=key, pcm=pcm if first else None, seek=seek,
                                      segment_size=3000, language_token=st.first_lang, token_budget=2)])
                eng.session_step(max_chunks=0)
                dt = time.perf_counter() - t
                while True:
                    _, active, queued = eng.session_step(max_chunks=4)
                    if active == 0 and queued == 0:
                        return dt
            long_ = np.tile(synth.chirp_clip(11, 60.0), 20)          # 20 minutes
            short = synth.chirp_clip(12, 30.5)
            admit(1, long_, 0, True)
            admit(2, short, 0, True)
            t_long = min(admit(1, long_, s, False) for s in (30000, 60000, 90000))
            t_short = min(admit(2, short, 0, False) for _ in range(3))
            print(f"admission: 20-min clip's later window {t_long * 1e3:.2f} ms, 30 s clip's {t_short * 1e3:.2f} ms")
            # (before the resident log-mel each later window re-uploaded 38 MB and recomputed the
            # 20-minute clip's 120 000-frame log-mel; the bound leaves room for timing noise)
            assert t_long < 4.0 * t_short + 5e-3, (t_long, t_short)
        finally:
            eng.session_end()
    finally:
        eng.close()


@pytest.mark.parametrize("beam", [1, 5])
def test_session_near_prompt_limits(beam):
    """the per-row prompt path near its limits — max_length 448 (the runner's),
    a <|startofprev|> prefix of 223 tokens (the seek loop's cap, 448 // 2 - 1, plus
    <|startofprev|>), windows that run to max_length (no budget) beside short ones: every
    window equals its decode alone (SelState::plen, pstride = n_text_ctx, beam lseq/lanc)."""
    d = D.TINY_TEST
    st = SpecialTokens.for_vocab(d.n_vocab)
    eng = WhisperEngine(d, device=0, max_batch=3)
    try:
        eng.load_weights(weights.random_weights(d, seed=31, emb_std=0.5))
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=448, beam_size=beam)
        wins = []
        for i in range(4):
            pcm = synth.chirp_clip(950 + i, 30.0)
            n_pre = (223, 223, 40, 0)[i]
            prefix = [st.sot_prev] + [200 + (17 * i + 5 * j) % 400 for j in range(n_pre)] if n_pre else None
            wins.append(dict(tag=i, pcm=pcm, seek=0, segment_size=3000, language_token=st.first_lang + i,
                             prefix=prefix, token_budget=(0, 12, 0, 30)[i]))
        got = _run_session(eng, cfg, wins, add_in=(0.5, 1.0))
        _compare(eng, cfg, wins, got)
        print("near-limit windows: prompt", [len(w["prefix"] or []) + 3 for w in wins], "sampled",
              [len(got[w["tag"]].tokens) for w in wins])
    finally:
        eng.close()
