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
