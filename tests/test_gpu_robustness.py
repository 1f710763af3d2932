"""GPU robustness: decoder row counts at every skinny-GEMM grouping boundary, and rows
whose logits are all NaN (no token can win the argmax).

The row-count test answers VERDICT r2 item 2: round 2 saw one illegal memory access in
the 32-row eager decoder step (gpurun_out/r02_ao) while the skinny GEMM's hi/lo row
grouping was being changed, in a tree that was never committed; these counts cover
every (grid z, MT) combination the committed launcher can pick."""
import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth, weights
from open_speech_amd.engine import DecodeConfig, WhisperEngine
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

pytestmark = pytest.mark.gpu


def test_decoder_row_group_boundaries_match_fp16_oracle():
    """31, 32, 33, 64 and 65 hi/lo decoder rows (skinny GEMM: one 64-row group with
    MT 2; 32-row groups on grid z = 2; z = 3 with a 1-row last group), eager steps with
    the logits dump (the r02_ao path), two clips alternating: every window's first 4
    steps' logits within 2e-2 of the fp16 oracle (the same bar as the 1-row test), its
    ids equal to the oracle's, and every copy of a clip identical to the others at every
    row count (bit-exact logits)."""
    from oracle import decode as odec
    from oracle.model import WhisperOracle
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=1234, emb_std=0.5)
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    cfg = DecodeConfig(suppress_tokens=sup, max_length=48)
    pcms = [synth.chirp_clip(11, 30.0), synth.chirp_clip(12, 30.0)]
    eng = WhisperEngine(d, device=0, max_batch=65)
    ref, enc0 = {}, {}
    try:
        eng.load_weights(w)
        orc = WhisperOracle(d, w, fp16=True)
        form = 0
        for n in (31, 32, 33, 64, 65):
            eng.log_mel([pcms[i % 2] for i in range(n)])
            eng.encode([(i, 0, 3000) for i in range(n)])
            outs = eng.decode(n, cfg, dump_steps=4)
            for k in range(2):
                enc = eng.encoder_output(k)
                if k not in enc0:
                    enc0[k] = enc
                if (form, k) not in ref:
                    ref[form, k] = odec.greedy_from_encoder(orc, orc.cross_kv(enc), st, keep_logits=4,
                                                            opts=odec.DecodeOptions(suppress_tokens=sup, max_length=48))
                np.testing.assert_array_equal(enc, enc0[k], err_msg=f"encoder output of clip {k} at {n} windows")
                for i in range(4):
                    np.testing.assert_allclose(outs[k].logits[i], ref[form, k].step_logits[i], atol=2e-2, rtol=0,
                                               err_msg=f"{n} rows, clip {k}, step {i}")
                assert outs[k].tokens == ref[form, k].tokens, (n, k)
                for j in range(k, n, 2):
                    assert outs[j].tokens == outs[k].tokens, (n, j)
                    np.testing.assert_array_equal(outs[j].logits, outs[k].logits, err_msg=f"{n} rows, window {j}")
    finally:
        eng.close()


@pytest.fixture(scope="module")
def nan_engine():
    """Micro dims with a NaN final-LayerNorm gain: every logit of every step is NaN."""
    d = D.MICRO_TEST
    w = weights.random_weights(d, seed=7, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=8)
    eng.load_weights(w)
    g = np.asarray(w["dec.lnpost.g"], np.float32).copy()
    eng.set_weight("dec.lnpost.g", np.full_like(g, np.nan))
    yield d, eng, w
    eng.close()


@pytest.mark.parametrize("mode", ["greedy_detect", "greedy_lang", "beam5", "sampling", "greedy_graph_rows",
                                  "greedy_b1", "greedy_b1_lang"])
def test_nan_logits_end_rows_without_fault(nan_engine, mode):
    """an all-NaN row never produces a winner (a NaN never beats the argmax
    seed {-inf, INT_MAX}).  Greedy, sampling and the language argmax must end the row
    with <|endoftext|> (as beam_update does for INT_MAX candidates) instead of using the
    id: no out-of-range token is emitted, embedded or used to index the logits, and the
    context stays usable."""
    d, eng, _ = nan_engine
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    kw = dict(suppress_tokens=sup, max_length=40)
    n = 3
    if mode == "greedy_lang":
        kw["language_token"] = st.first_lang
    elif mode == "beam5":
        kw["beam_size"] = 5
    elif mode == "sampling":
        kw.update(temperature=0.7, best_of=2, seed=3)
    elif mode == "greedy_graph_rows":
        n = 8                      # decode graph (no dump), 8 rows
    elif mode.startswith("greedy_b1"):
        n = 1                      # one row: the selection fused into the logits GEMM
        if mode.endswith("lang"):
            kw["language_token"] = st.first_lang
    clips = [synth.chirp_clip(70 + i, 30.0) for i in range(n)]
    outs = eng.transcribe_batch(clips, DecodeConfig(**kw))
    for o in outs:
        assert o.tokens == [], o.tokens
        assert st.first_lang <= o.language < st.first_lang + st.n_langs
    # the context still decodes (no fault left behind)
    again = eng.transcribe_batch(clips[:1], DecodeConfig(suppress_tokens=sup, max_length=24))
    assert again[0].tokens == []


def test_context_usable_after_nan_rows(nan_engine):
    """After NaN rows, restoring the weight gives the normal decode of a fresh engine."""
    d, eng, w = nan_engine
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    cfg = DecodeConfig(suppress_tokens=sup, max_length=32)
    clip = synth.chirp_clip(80, 30.0)
    eng.transcribe_batch([clip], cfg)
    eng.set_weight("dec.lnpost.g", np.asarray(w["dec.lnpost.g"], np.float32))
    got = eng.transcribe_batch([clip], cfg)[0]
    fresh = WhisperEngine(d, device=0, max_batch=1)
    try:
        fresh.load_weights(w)
        want = fresh.transcribe_batch([clip], cfg)[0]
    finally:
        fresh.close()
    assert got.tokens == want.tokens and got.sum_logprob == want.sum_logprob
    assert all(0 <= t < d.n_vocab for t in got.tokens)


def test_batch1_fused_selection_equals_select_kernel():
    """One decoder row selects its token in the logits GEMM's epilogue (SelFuse); two or
    more rows use select_kernel.  The same window alone and in a 2-window batch: ids,
    language and no-speech prob identical, sum_logprob equal up to the order of the
    log-sum-exp merges (811 workgroup records vs 16 slices); with a token budget (the
    finaliser's <|endoftext|> read-back) and with the logits dump (eager steps)."""
    d = D.TINY_TEST
    w = weights.random_weights(d, seed=1234, emb_std=0.5)
    eng = WhisperEngine(d, device=0, max_batch=2)
    try:
        eng.load_weights(w)
        sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
        clips = [synth.chirp_clip(90, 30.0), synth.chirp_clip(91, 17.0)]
        for budget in (None, (7, 11)):
            cfg = DecodeConfig(suppress_tokens=sup, max_length=96, token_budget=budget)
            both = eng.transcribe_batch(clips, cfg)
            for i, c in enumerate(clips):
                one_cfg = DecodeConfig(suppress_tokens=sup, max_length=96,
                                       token_budget=None if budget is None else (budget[i],))
                one = eng.transcribe_batch([c], one_cfg)[0]
                assert one.tokens == both[i].tokens, (budget, i)
                assert one.language == both[i].language
                assert abs(one.no_speech_prob - both[i].no_speech_prob) < 1e-5
                assert abs(one.sum_logprob - both[i].sum_logprob) <= 1e-4 * (len(one.tokens) + 1)
                if budget is not None:
                    assert len(one.tokens) == budget[i]
        eng.log_mel(clips[:1])
        eng.encode([(0, 0, 3000)])
        cfg = DecodeConfig(suppress_tokens=sup, max_length=96)
        dumped = eng.decode(1, cfg, dump_steps=3)[0]
        assert dumped.tokens == eng.transcribe_batch(clips[:1], cfg)[0].tokens
    finally:
        eng.close()
