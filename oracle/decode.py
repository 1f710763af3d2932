"""ORACLE (test infrastructure only) — greedy Whisper decoding with the logits
processors faster-whisper asks CTranslate2 to apply (upstream, not vendored).

Options mirror faster-whisper 1.2.1's ``transcribe`` defaults as called by the
reference (``src/backends/faster_whisper.py:235-245``) with ``beam_size=1`` for the
greedy parity mode: ``suppress_blank=True``, ``suppress_tokens=[-1]`` (expanded by
``get_suppressed_tokens``), ``without_timestamps=False``,
``max_initial_timestamp=1.0`` (index 50), ``max_length=448`` positions.

The processors follow openai-whisper's ``SuppressBlank``, ``SuppressTokens`` and
``ApplyTimestampRules`` (in-container restatement: transformers
``generation/logits_process.py:1816,1869,1909``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

NEG_INF = -np.inf


def log_softmax(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float64)
    m = np.max(x)
    return x - (m + np.log(np.sum(np.exp(x - m))))


def logsumexp(x: np.ndarray) -> float:
    x = x.astype(np.float64)
    m = np.max(x)
    if not np.isfinite(m):
        return float(m)
    return float(m + np.log(np.sum(np.exp(x - m))))


# the model's maximum decoder length: previous text keeps its last 448 // 2 - 1 tokens
# whatever max_length a call uses (faster-whisper get_prompt uses self.max_length = 448)
MODEL_MAX_LENGTH = 448


@dataclass
class DecodeOptions:
    suppress_blank: bool = True
    suppress_tokens: tuple = ()
    without_timestamps: bool = False
    max_initial_timestamp_index: int = 50
    max_length: int = 448


def process_logits(logits: np.ndarray, sampled: list, st, opts: DecodeOptions) -> np.ndarray:
    """Apply the logits filters for the next token given the tokens sampled so far."""
    x = logits.astype(np.float64).copy()
    n = len(sampled)
    tb = st.timestamp_begin
    if opts.suppress_blank and n == 0:
        x[[st.blank, st.eot]] = NEG_INF
    if len(opts.suppress_tokens):
        x[list(opts.suppress_tokens)] = NEG_INF
    if not opts.without_timestamps:
        x[st.no_timestamps] = NEG_INF
        last = n >= 1 and sampled[-1] >= tb
        pen = n < 2 or sampled[-2] >= tb
        if last:
            if pen:
                x[tb:] = NEG_INF
            else:
                x[:st.eot] = NEG_INF
        ts = [t for t in sampled if t >= tb]
        if ts:
            tl = ts[-1] if (last and not pen) else ts[-1] + 1
            x[tb:tl] = NEG_INF
        if n == 0:
            x[:tb] = NEG_INF
            if opts.max_initial_timestamp_index is not None:
                x[tb + opts.max_initial_timestamp_index + 1:] = NEG_INF
        lp = log_softmax(x)
        if logsumexp(lp[tb:]) > np.max(lp[:tb]):
            x[:tb] = NEG_INF
    return x


@dataclass
class WindowResult:
    tokens: list
    sum_logprob: float
    no_speech_prob: float
    language: int
    step_logits: list = field(default_factory=list)   # raw fp32 logits per generated step
    prompt_logits: list = field(default_factory=list)
    hypotheses: list = field(default_factory=list)    # beam: every finished (tokens, raw, normalised score), in order


def detect_language(raw_sot_logits: np.ndarray, st) -> int:
    lang = raw_sot_logits[st.first_lang:st.first_lang + st.n_langs]
    return st.first_lang + int(np.argmax(lang))


def no_speech_prob(raw_sot_logits: np.ndarray, st) -> float:
    return float(np.exp(log_softmax(raw_sot_logits)[st.no_speech]))


def greedy_window(oracle, mel_window, st, *, language=None, task=None, prev_tokens=(),
                  opts: DecodeOptions = DecodeOptions(), keep_logits: int = 0) -> WindowResult:
    """Encode one 30 s window and decode greedily (faster-whisper get_prompt + CT2 generate)."""
    enc = oracle.encode(mel_window)
    xkv = oracle.cross_kv(enc)
    return greedy_from_encoder(oracle, xkv, st, language=language, task=task, prev_tokens=prev_tokens,
                               opts=opts, keep_logits=keep_logits)


def greedy_from_encoder(oracle, xkv, st, *, language=None, task=None, prev_tokens=(),
                        opts: DecodeOptions = DecodeOptions(), keep_logits: int = 0) -> WindowResult:
    task = st.transcribe if task is None else task
    cache = oracle.new_cache()
    prompt = []
    if prev_tokens:
        prompt.append(st.sot_prev)
        prompt.extend(list(prev_tokens)[-(MODEL_MAX_LENGTH // 2 - 1):])
    sot_index = len(prompt)
    prompt.append(st.sot)
    pos = 0
    prompt_logits = []
    for t in prompt:                      # feed up to and including SOT
        lg = oracle.decoder_step(t, pos, cache, xkv)
        pos += 1
    raw_sot = lg
    prompt_logits.append(raw_sot)
    lang = detect_language(raw_sot, st) if language is None else language
    nsp = no_speech_prob(raw_sot, st)
    rest = [lang, task] + ([st.no_timestamps] if opts.without_timestamps else [])
    for t in rest:
        lg = oracle.decoder_step(t, pos, cache, xkv)
        pos += 1
    prompt_len = len(prompt) + len(rest)
    sampled: list = []
    sum_lp = 0.0
    step_logits = []
    while True:
        if keep_logits and len(step_logits) < keep_logits:
            step_logits.append(lg.copy())
        x = process_logits(lg, sampled, st, opts)
        nxt = int(np.argmax(x))
        sum_lp += float(log_softmax(x)[nxt])
        if nxt == st.eot:
            break
        sampled.append(nxt)
        if prompt_len + len(sampled) >= opts.max_length:
            break
        lg = oracle.decoder_step(nxt, pos, cache, xkv)
        pos += 1
    del sot_index
    return WindowResult(tokens=sampled, sum_logprob=sum_lp, no_speech_prob=nsp, language=lang,
                        step_logits=step_logits, prompt_logits=prompt_logits)


# ---------------------------------------------------------------------------
# Beam search — restated from CTranslate2's ``BeamSearch::search`` (upstream
# ``src/decoding.cc``, not vendored and not installed here; faster-whisper 1.2.1
# calls it with ``beam_size=5, patience=1, length_penalty=1, num_hypotheses=1``
# from ``generate_with_fallback`` for the reference's ``beam_size=5``,
# ``src/backends/faster_whisper.py:237``).  PARITY UNPINNED: no CTranslate2 build or
# beam-search fixture exists in this container, so this restatement (not CT2
# output) is the checker for the HIP beam path.  Rules restated:
#   * the first sampled step expands only the single prompt hypothesis;
#   * candidates = top 2*beam of (cumulative score + processed log-prob) over
#     beam x vocab, ordered by score desc, flat index (beam*V + token) asc;
#   * of the first ``beam`` candidates, an <|endoftext|> one (or any one at the
#     last step) is registered as a finished hypothesis with its cumulative score
#     and its slot is refilled by the next non-EOT candidate from ranks >= beam;
#   * stop when the last step is reached, or the rank-0 candidate finished this
#     step and >= num_hypotheses are finished, or >= round(beam*patience) are;
#   * result = the finished hypothesis with the highest score / len**length_penalty
#     (len = its token count without EOT; first registered wins ties).
# ---------------------------------------------------------------------------
@dataclass
class BeamOptions:
    beam_size: int = 5
    patience: float = 1.0
    length_penalty: float = 1.0
    num_hypotheses: int = 1
    # the length a finished score is normalised by counts its <|endoftext|> (transformers'
    # convention, generated_len = cur_len + 1 - prompt_len, generation/utils.py:3182); only
    # the transformers cross-check sets it (tools/make_hf_pins.py)
    length_counts_eot: bool = False


def _norm_score(score: float, n: int, length_penalty: float) -> float:
    if n == 0:
        return -np.inf if length_penalty != 0 else score
    return score / (float(n) ** length_penalty)


def beam_from_encoder(oracle, xkv, st, *, language=None, task=None, prev_tokens=(),
                      opts: DecodeOptions = DecodeOptions(), beam: BeamOptions = BeamOptions()) -> WindowResult:
    import copy

    task = st.transcribe if task is None else task
    cache = oracle.new_cache()
    prompt = []
    if prev_tokens:
        prompt.append(st.sot_prev)
        prompt.extend(list(prev_tokens)[-(MODEL_MAX_LENGTH // 2 - 1):])
    prompt.append(st.sot)
    pos = 0
    for t in prompt:
        lg = oracle.decoder_step(t, pos, cache, xkv)
        pos += 1
    raw_sot = lg
    lang = detect_language(raw_sot, st) if language is None else language
    nsp = no_speech_prob(raw_sot, st)
    rest = [lang, task] + ([st.no_timestamps] if opts.without_timestamps else [])
    for t in rest:
        lg = oracle.decoder_step(t, pos, cache, xkv)
        pos += 1
    prompt_len = len(prompt) + len(rest)
    K = beam.beam_size
    V = lg.shape[0]
    max_cand = int(round(K * beam.patience))
    alive = [([], 0.0, cache, lg)]        # (tokens, cumulative score, kv cache, next-token logits)
    finished = []                         # (normalised, raw score, tokens)
    n = 0
    while True:
        is_last = prompt_len + n + 1 >= opts.max_length
        scores = []
        for k, (seq, cum, _, logit) in enumerate(alive):
            x = process_logits(logit, seq, st, opts)
            lp = log_softmax(x).astype(np.float32)
            scores.append(np.float32(cum) + lp)
        flat = np.concatenate(scores)
        order = np.lexsort((np.arange(flat.size), -flat.astype(np.float64)))[:2 * K]
        cands = [(float(flat[i]), int(i) // V, int(i) % V) for i in order]
        chosen, sec, top_fin = [], K, False
        for k in range(K):
            s, q, tok = cands[k]
            nb = k
            if tok == st.eot or is_last:
                if k == 0:
                    top_fin = True
                toks = list(alive[q][0]) + ([] if tok == st.eot else [tok])
                n_len = len(toks) + (1 if beam.length_counts_eot and tok == st.eot else 0)
                finished.append((_norm_score(s, n_len, beam.length_penalty), s, toks))
                for j in range(sec, 2 * K):
                    if cands[j][2] != st.eot:
                        nb, sec = j, j + 1
                        break
            chosen.append(cands[nb])
        if is_last or (top_fin and len(finished) >= beam.num_hypotheses) or len(finished) >= max_cand:
            break
        nxt = []
        for s, q, tok in chosen:
            seq, _, cch, _ = alive[q]
            c2 = copy.deepcopy(cch)
            logit = oracle.decoder_step(tok, pos, c2, xkv)
            nxt.append((list(seq) + [tok], s, c2, logit))
        alive = nxt
        pos += 1
        n += 1
    best = finished[0]
    for f in finished[1:]:
        if f[0] > best[0]:
            best = f
    return WindowResult(tokens=best[2], sum_logprob=best[1], no_speech_prob=nsp, language=lang,
                        hypotheses=[(f[2], f[1], f[0]) for f in finished])


# ---------------------------------------------------------------------------
# Sampling at temperature > 0 — faster-whisper's sampling branch of
# ``generate_with_fallback`` [upstream] (``beam_size=1, num_hypotheses=best_of,
# sampling_topk=0, sampling_temperature=T``).  The device draws every token by the
# Gumbel-max trick on a counter hash (``gumbel_noise`` in csrc/decode.hip), so a
# draw is reproducible from (seed, decoder row, step, token); this restates that
# draw bit for bit in float32.  PARITY UNPINNED against CTranslate2, whose RNG
# stream cannot be reproduced; what is pinned is the draw rule: argmax over the
# rule-masked logits of x / T + G is a sample of softmax(x / T) over those tokens.
# ---------------------------------------------------------------------------
_M64 = 0xFFFFFFFFFFFFFFFF


def gumbel_noise(seed: int, row: int, step: int, v: np.ndarray) -> np.ndarray:
    """float32 Gumbel(0, 1) noise for tokens ``v`` (splitmix64 finaliser, 23-bit uniform)."""
    v = np.asarray(v, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = (seed + 0x9E3779B97F4A7C15 * (row + 1) + 0xD1B54A32D192ED03 * (step + 1)) & _M64
        z = np.uint64(base) + np.uint64(0x94D049BB133111EB) * (v + np.uint64(1))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = ((z >> np.uint64(41)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)
    return -np.log(-np.log(u))


def sample_token(x_processed: np.ndarray, inv_temp: float, seed: int, row: int, step: int) -> int:
    """One draw from softmax(x / T) over the finite (kept) entries of the processed logits;
    ties go to the lowest token id."""
    idx = np.nonzero(np.isfinite(x_processed))[0]
    key = x_processed[idx].astype(np.float32) * np.float32(inv_temp) + gumbel_noise(seed, row, step, idx)
    return int(idx[int(np.argmax(key))])
