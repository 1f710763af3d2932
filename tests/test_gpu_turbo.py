"""whisper-large-v3-turbo (the benchmarked model, BASELINE configs[1..3]) on the GPU
against the fp32 transformers golden (tools/make_golden.py gen_turbo: the same
hash-initialised weights the GPU regenerates with init_random(seed=0), the same
30 s chirp clip).

North-star bar: greedy token ids bit-exact; logits within 1e-3.  The norm is stated
here: the log-softmax of the RAW logits (before the logits rules), compared in
float64, max |Δ| over the whole vocabulary for the first 4 sampled steps and every
32nd step after them, and over 288 tokens per step (the step's golden top-32 plus a
fixed sample of 256 token ids) for every other step.  A divergence of ids FAILS the
test; the failure message carries the golden top-2 margin at the divergence so a
near-tie can be told from a bug.

Beam search width 5 (the reference's decoding, src/backends/faster_whisper.py:237)
is checked against tests/golden/turbo_beam5.npz: the oracle's CTranslate2-BeamSearch
restatement driven by the fp32 transformers decoder on the same weights and clip
(tools/make_golden.py gen_turbo_beam), 93 sampled positions.

The i.i.d. weights above decode few distinct ids (timestamp pairs, repeated tokens), so
their id checks barely discriminate.  The "text" goldens (tests/golden/turbo_text.npz,
weights.text_positional) decode ~440 distinct ids in 445 steps on each of three clips
with a golden top-2 margin >= 0.04 at every step; their ids are checked exactly, with the
same 1e-3 log-softmax bar, and beam 5 on them.
"""
import os

import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth
from open_speech_amd.engine import DecodeConfig, WhisperEngine
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
LSM_TOL = 1e-3
NEAR_TIE = 2e-3


def lse(x):
    x = np.asarray(x, np.float64)
    m = x.max()
    return m + np.log(np.exp(x - m).sum())


@pytest.fixture(scope="module")
def turbo():
    d = D.LARGE_V3_TURBO
    eng = WhisperEngine(d, device=0, max_batch=64)
    eng.init_random(seed=0)
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    yield d, eng, sup
    eng.close()


def first_divergence(got, want, margins):
    n = min(len(got), len(want))
    for k in range(n):
        if got[k] != want[k]:
            return k
    return None if len(got) == len(want) else n


def test_turbo_greedy_matches_fp32_golden(turbo):
    d, eng, sup = turbo
    z = np.load(os.path.join(GOLD, "turbo_model.npz"))
    eng.log_mel([synth.chirp_clip(0, 30.0)])
    eng.encode([(0, 0, 3000)])
    enc = eng.encoder_output(0)
    # encoder output (fp16 storage) vs fp32
    rows = z["enc_rows"]
    assert np.abs(enc[rows] - z["enc"]).max() < 1e-2
    np.testing.assert_allclose(np.linalg.norm(enc.astype(np.float64), axis=1), z["enc_rownorm"], rtol=1e-3)
    want = z["ids"].tolist()
    out = eng.decode(1, DecodeConfig(suppress_tokens=sup), dump_steps=len(want) + 1)[0]
    assert out.language == int(z["language"])
    assert abs(out.no_speech_prob - float(z["no_speech_prob"])) < 1e-3
    k = first_divergence(out.tokens, want, z["margins"])
    n_ok = len(want) + 1 if k is None else k + 1   # steps whose history matched (logits comparable)
    # log-softmax of the raw logits
    full_at = {int(t): i for i, t in enumerate(z["full_steps"])}
    errs, n_full = [], 0
    for s in range(min(n_ok, len(z["lse"]))):
        g = out.logits[s].astype(np.float64)
        lg = lse(g)
        if s in full_at:
            ref = z["full_logits"][full_at[s]].astype(np.float64) - z["lse"][s]
            errs.append(np.abs((g - lg) - ref).max())
            n_full += 1
        ids = z["sub_ids"][s]
        errs.append(np.abs((g[ids] - lg) - (z["sub_vals"][s].astype(np.float64) - z["lse"][s])).max())
    print(f"turbo: {len(out.tokens)} ids, divergence at {k}, log-softmax max |d| {max(errs):.3e} over "
          f"{min(n_ok, len(z['lse']))} steps ({n_full} of them over the full vocabulary)")
    assert n_full >= 15
    assert max(errs) <= LSM_TOL, max(errs)
    if k is not None:
        margin = float(z["margins"][k]) if k < len(z["margins"]) else float("nan")
        pytest.fail(f"ids identical for {k} steps, then diverge: golden top-2 margin {margin:.4g} "
                    f"({'a near-tie' if margin < NEAR_TIE else 'NOT a near-tie'})")


def test_turbo_batch64_equals_single_windows(turbo):
    """BASELINE configs[2]: 64 x 30 s windows in one batch; windows 0, 31 and 63 decode
    exactly as when run alone, and window 0 (the golden clip) reproduces the golden ids."""
    d, eng, sup = turbo
    z = np.load(os.path.join(GOLD, "turbo_model.npz"))
    clips = [synth.chirp_clip(i, 30.0) for i in range(64)]
    cfg = DecodeConfig(suppress_tokens=sup)
    batch = eng.transcribe_batch(clips, cfg)
    assert len(batch) == 64
    for i in (0, 31, 63):
        one = eng.transcribe_batch([clips[i]], cfg)[0]
        assert one.tokens == batch[i].tokens, i
        assert one.language == batch[i].language
        # 1 row vs 64 rows: the logits GEMM kernel differs (skinny vs the 64-row wide
        # kernel), so the fp32 sums differ in accumulation order only
        assert abs(one.sum_logprob - batch[i].sum_logprob) <= 1e-4 * (len(one.tokens) + 1)
    want = z["ids"].tolist()
    k = first_divergence(batch[0].tokens, want, z["margins"])
    assert k is None or float(z["margins"][k]) < NEAR_TIE, (k, float(z["margins"][k]))


@pytest.mark.parametrize("n", [3, 4, 9])
def test_turbo_encoder_few_windows_equal_single(turbo, n):
    """The few-window encoders (streaming calls, session admissions) pick other GEMM tiles
    than one window does — at 3-4 windows the half-width 256 x 128 tile for qkv (head-major
    epilogue), fc1 (GELU) and the fp32 residual GEMMs, at 9 the 8-phase 256 tile (DESIGN
    §5.12) — and every window's encoder output is bit-identical to the window encoded alone."""
    d, eng, sup = turbo
    clips = [synth.chirp_clip(40 + i, 30.0 - 2.5 * i) for i in range(n)]
    nf = eng.log_mel(clips)
    wins = [(i, 0, min(3000, nf[i] - 1)) for i in range(n)]
    eng.encode(wins)
    many = [eng.encoder_output(k) for k in range(n)]
    for k in range(n):
        eng.log_mel([clips[k]])
        eng.encode([(0, 0, wins[k][2])])
        assert np.array_equal(eng.encoder_output(0), many[k]), k


def test_turbo_beam5_matches_fp32_golden(turbo):
    """Beam 5 on the benchmarked model: ids identical to the fp32 golden, cumulative
    log-prob within 1e-4 per token (+1e-3 relative), language and no-speech prob equal."""
    d, eng, sup = turbo
    z = np.load(os.path.join(GOLD, "turbo_beam5.npz"))
    eng.log_mel([synth.chirp_clip(0, 30.0)])
    eng.encode([(0, 0, 3000)])
    cfg = DecodeConfig(suppress_tokens=sup, max_length=int(z["max_length"]), beam_size=5)
    out = eng.decode(1, cfg)[0]
    want = z["ids"].tolist()
    assert out.language == int(z["language"])
    assert abs(out.no_speech_prob - float(z["no_speech_prob"])) < 1e-3
    k = first_divergence(out.tokens, want, None)
    assert k is None, f"beam ids diverge at step {k}: gpu {out.tokens[k:k + 4]} vs golden {want[k:k + 4]}"
    ref = float(z["sum_logprob"])
    assert abs(out.sum_logprob - ref) <= 1e-4 * (len(want) + 1) + 1e-3 * abs(ref), (out.sum_logprob, ref)


def test_turbo_beam5_batch64_equals_single_windows(turbo):
    """Beam 5 over a 64-window batch (320 decoder rows: the tiled split-K projections,
    the 320-row logits GEMM, the MFMA beam cross-attention): windows 0, 31 and 63 give
    the ids of their single-window runs, window 0 the golden ids."""
    d, eng, sup = turbo
    z = np.load(os.path.join(GOLD, "turbo_beam5.npz"))
    clips = [synth.chirp_clip(i, 30.0) for i in range(64)]
    cfg = DecodeConfig(suppress_tokens=sup, max_length=int(z["max_length"]), beam_size=5)
    batch = eng.transcribe_batch(clips, cfg)
    assert len(batch) == 64
    for i in (0, 31, 63):
        one = eng.transcribe_batch([clips[i]], cfg)[0]
        assert one.tokens == batch[i].tokens, i
        assert one.language == batch[i].language
        # 5 rows (skinny split-K) vs 320 rows (tiled split-K): accumulation order only
        assert abs(one.sum_logprob - batch[i].sum_logprob) <= 1e-4 * (len(one.tokens) + 1) + \
            1e-4 * abs(one.sum_logprob), i
    assert batch[0].tokens == z["ids"].tolist()


# --------------------------------------------------------------------------- text goldens
# tests/golden/turbo_text.npz (tools/make_golden.py gen_turbo_text): the same model with a
# constructed positional table (construct_audio_table, stored as pos_table): each position
# leans to a pseudo-random text token, and at most positions to a second token as well, with
# the clip's audio (through the cross-attention) deciding between them.  Three spectrally
# distinct clips (chirp, 440 Hz tone, white noise); every pair differs at >= 100 of the 445
# ids; the golden top-2 margins are in meta.json "turbo_text".  Free-running ids must be
# identical over all 445 steps; a decoder that copies its previous token, drops a layer or
# ignores the encoder cannot pass.
TEXT = os.path.join(GOLD, "turbo_text.npz")


def _meta(key):
    import json
    return json.load(open(os.path.join(GOLD, "meta.json")))[key]


@pytest.fixture(scope="module")
def turbo_text():
    d = D.LARGE_V3_TURBO
    m = _meta("turbo_text")
    z = np.load(TEXT)
    eng = WhisperEngine(d, device=0, max_batch=8)
    eng.init_random(seed=m["seed"], text_pos=m["text_pos"])
    # the constructed, audio-dependent positional table (tools/make_golden.py construct_audio_table)
    eng.set_weight("dec.pos", z["pos_table"])
    sup = get_suppressed_tokens(WhisperTokenizer(d.n_vocab), [-1])
    yield d, eng, sup, z, m
    eng.close()


TEXT_CLIPS = ["chirp0", "tone", "noise"]


def _text_clip(name):
    return {"chirp0": lambda: synth.chirp_clip(0, 30.0), "tone": lambda: synth.tone_clip(30.0),
            "noise": lambda: synth.noise_clip(5, 30.0)}[name]()


def test_turbo_text_golden_depends_on_audio(turbo_text):
    """the golden ids are a function of the audio — every pair of the
    three clips differs at >= 100 of the 445 positions (a decoder whose cross-attention
    ignored the encoder would emit one sequence for all three)."""
    d, eng, sup, z, m = turbo_text
    for i, a in enumerate(TEXT_CLIPS):
        for b in TEXT_CLIPS[i + 1:]:
            x, y = z[a + "/ids"], z[b + "/ids"]
            assert len(x) == len(y) == 445
            assert int((x != y).sum()) >= 100, (a, b)


def _lsm_err(out_logits, z, pre, n_steps):
    full_at = {int(t): i for i, t in enumerate(z[pre + "full_steps"])}
    errs, n_full = [], 0
    for s in range(n_steps):
        g = out_logits[s].astype(np.float64)
        lg = lse(g)
        if s in full_at:
            ref = z[pre + "full_logits"][full_at[s]].astype(np.float64) - z[pre + "lse"][s]
            errs.append(np.abs((g - lg) - ref).max())
            n_full += 1
        ids = z[pre + "sub_ids"][s]
        errs.append(np.abs((g[ids] - lg) - (z[pre + "sub_vals"][s].astype(np.float64) - z[pre + "lse"][s])).max())
    return max(errs), n_full


@pytest.mark.parametrize("clip", TEXT_CLIPS)
def test_turbo_text_greedy_ids_exact(turbo_text, clip):
    """Varied-text golden, one window: every one of the 445 greedy ids identical, language
    and no-speech prob equal, and the log-softmax of the raw logits within 1e-3 (over the
    whole vocabulary at the first 4 steps, and every 32nd for chirp0; over 288 tokens per
    step at every step)."""
    d, eng, sup, z, m = turbo_text
    pre = clip + "/"
    eng.log_mel([_text_clip(clip)])
    eng.encode([(0, 0, 3000)])
    enc = eng.encoder_output(0)
    np.testing.assert_allclose(np.linalg.norm(enc.astype(np.float64), axis=1), z[pre + "enc_rownorm"], rtol=1e-3)
    want = z[pre + "ids"].tolist()
    assert len(set(want)) >= 150 and len(want) >= 300   # the golden itself is discriminative (and see
                                                        # test_turbo_text_golden_depends_on_audio)
    out = eng.decode(1, DecodeConfig(suppress_tokens=sup), dump_steps=len(want) + 1)[0]
    assert out.language == int(z[pre + "language"])
    assert abs(out.no_speech_prob - float(z[pre + "no_speech_prob"])) < 1e-3
    k = first_divergence(out.tokens, want, None)
    n_ok = len(want) + 1 if k is None else k + 1
    err, n_full = _lsm_err(out.logits, z, pre, min(n_ok, len(z[pre + "lse"])))
    print(f"turbo text {clip}: {len(out.tokens)} ids ({len(set(out.tokens))} distinct), divergence at {k}, "
          f"log-softmax max |d| {err:.3e} ({n_full} full-vocabulary steps), golden min margin "
          f"{float(z[pre + 'margins'].min()):.3g}")
    assert k is None, (f"ids diverge at step {k}: gpu {out.tokens[k:k + 4]} vs golden {want[k:k + 4]}, golden "
                       f"top-2 margin {float(z[pre + 'margins'][k]):.4g}")
    assert err <= LSM_TOL, err
    assert abs(out.sum_logprob - float(z[pre + "sum_logprob"])) <= 1e-4 * (len(want) + 1)


def test_turbo_text_batch_equals_golden(turbo_text):
    """The three clips in one batch (3 decoder rows): every window's ids equal the golden."""
    d, eng, sup, z, m = turbo_text
    names = TEXT_CLIPS
    outs = eng.transcribe_batch([_text_clip(n) for n in names], DecodeConfig(suppress_tokens=sup))
    for n, o in zip(names, outs):
        assert o.tokens == z[n + "/ids"].tolist(), n


def test_turbo_text_beam5_matches_golden(turbo_text):
    """Beam 5 (the reference's decoding) on the varied-text weights: ids identical to the
    oracle's CTranslate2-BeamSearch restatement over the fp32 transformers decoder,
    cumulative log-prob within 1e-4 per token."""
    d, eng, sup, z, m = turbo_text
    eng.log_mel([_text_clip("chirp0")])
    eng.encode([(0, 0, 3000)])
    cfg = DecodeConfig(suppress_tokens=sup, max_length=int(z["beam5/max_length"]), beam_size=5)
    out = eng.decode(1, cfg)[0]
    want = z["beam5/ids"].tolist()
    assert len(set(want)) >= 60
    assert out.language == int(z["beam5/language"])
    k = first_divergence(out.tokens, want, None)
    assert k is None, f"beam ids diverge at step {k}: gpu {out.tokens[k:k + 4]} vs golden {want[k:k + 4]}"
    ref = float(z["beam5/sum_logprob"])
    assert abs(out.sum_logprob - ref) <= 1e-4 * (len(want) + 1) + 1e-3 * abs(ref), (out.sum_logprob, ref)
