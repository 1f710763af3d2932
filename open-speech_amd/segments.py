"""Window scheduling and segment assembly (faster-whisper 1.2.1 ``generate_segments``,
upstream, not vendored), batched across clips.

For every clip the 30 s seek loop of faster-whisper runs unchanged — window k+1
depends on window k's last timestamp and (with ``condition_on_previous_text``) its
tokens — but the windows of DIFFERENT clips that are due at the same time are
encoded and decoded together on the GPU (grouped by prompt length, since every
window of one decode call shares its prompt length).

Semantics restated (beam search width ``beam_size`` — 5 in the reference, 1 = greedy
for the parity mode — at temperature 0.0; the reference passes a scalar ``temperature``
at ``src/backends/faster_whisper.py:238``, so there is no fallback, and a request with
temperature > 0 takes faster-whisper's sampling branch: ``best_of`` samples per window,
the best kept, and the previous-text prompt reset when temperature > 0.5):
  content_frames = n_frames - 1; segment_size = min(3000, content_frames - seek)
  prompt = [<|startofprev|>] + previous_tokens[-223:] (if any) + [sot, lang, task]
  avg_logprob = sum_logprob / (len(tokens) + 1); compression_ratio of the window text
  skip window if no_speech_prob > 0.6 and avg_logprob < -1.0  (seek += segment_size)
  split at consecutive timestamp pairs; single timestamp ending -> seek += segment_size,
  else seek += last_timestamp_position * 2; drop segments with start == end or blank text
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .dims import HOP_LENGTH, INPUT_STRIDE, N_FRAMES, TIME_PRECISION
from .engine import DecodeConfig
from .tokenizer import WhisperTokenizer, compression_ratio

FRAME_SEC = 0.01


@dataclass
class TranscribeOptions:
    task: str = "transcribe"
    language: str | None = None
    initial_prompt: str | None = None
    condition_on_previous_text: bool = True
    no_speech_threshold: float | None = 0.6
    log_prob_threshold: float | None = -1.0
    compression_ratio_threshold: float | None = 2.4
    suppress_blank: bool = True
    suppress_tokens: tuple = (-1,)
    without_timestamps: bool = False
    max_initial_timestamp: float = 1.0
    temperature: float = 0.0
    beam_size: int = 5             # faster-whisper / reference default (src/backends/faster_whisper.py:237)
    patience: float = 1.0
    length_penalty: float = 1.0
    best_of: int = 5               # faster-whisper default; used when temperature > 0
    prompt_reset_on_temperature: float = 0.5
    seed: int = 0
    # faster-whisper's max_new_tokens: a window's decode stops after this many sampled
    # tokens (max_length = prompt length + max_new_tokens, which may not exceed 448)
    max_new_tokens: int | None = None
    # bench-only length control (HipWhisperBackend(length_control=...)): random weights never emit
    # <|endoftext|>, so each window's decode is cut at ceil(rate * window seconds) + 2
    tokens_per_second: float | None = None

    def key(self):
        return (self.task, self.language, self.initial_prompt, self.condition_on_previous_text,
                self.without_timestamps, tuple(self.suppress_tokens), self.suppress_blank, self.beam_size,
                self.patience, self.length_penalty, self.temperature, self.best_of, self.tokens_per_second,
                self.max_new_tokens)


@dataclass
class Segment:
    id: int
    seek: int
    start: float
    end: float
    text: str
    tokens: list
    temperature: float
    avg_logprob: float
    compression_ratio: float
    no_speech_prob: float


@dataclass
class ClipResult:
    segments: list = field(default_factory=list)
    language: str = "en"
    duration: float = 0.0


def split_segments_by_timestamps(tokens: list, tb: int, time_offset: float, segment_size: int,
                                 segment_duration: float, seek: int):
    """faster-whisper ``_split_segments_by_timestamps`` (openai transcribe.py logic)."""
    current = []
    single_timestamp_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    consecutive = [i for i in range(len(tokens)) if i > 0 and tokens[i] >= tb and tokens[i - 1] >= tb]
    if consecutive:
        slices = list(consecutive)
        if single_timestamp_ending:
            slices.append(len(tokens))
        last_slice = 0
        for cur in slices:
            sliced = tokens[last_slice:cur]
            start_pos = sliced[0] - tb
            end_pos = sliced[-1] - tb
            current.append(dict(seek=seek, start=time_offset + start_pos * TIME_PRECISION,
                                end=time_offset + end_pos * TIME_PRECISION, tokens=sliced))
            last_slice = cur
        if single_timestamp_ending:
            seek += segment_size
        else:
            last_ts_pos = tokens[last_slice - 1] - tb
            seek += last_ts_pos * INPUT_STRIDE
    else:
        duration = segment_duration
        ts = [t for t in tokens if t >= tb]
        if ts and ts[-1] != tb:
            duration = (ts[-1] - tb) * TIME_PRECISION
        current.append(dict(seek=seek, start=time_offset, end=time_offset + duration, tokens=tokens))
        seek += segment_size
    return current, seek, single_timestamp_ending


@dataclass
class _ClipState:
    idx: int
    content_frames: int
    seek: int = 0
    all_tokens: list = field(default_factory=list)
    prompt_reset_since: int = 0
    lang_token: int | None = None
    done: bool = False
    result: ClipResult = field(default_factory=ClipResult)


def transcribe_clips(engine, pcm_list: list, opts: TranscribeOptions, tok: WhisperTokenizer,
                     suppress: tuple) -> list[ClipResult]:
    """Run the seek loop for a batch of int16 clips on one engine (all share `opts`)."""
    st = tok.special
    nf = engine.log_mel(pcm_list)
    lang_token = tok.language_token(opts.language) if (opts.language and opts.task == "transcribe") else None
    init_tokens = tok.encode(" " + opts.initial_prompt.strip()) if opts.initial_prompt else []
    states = []
    for i, n in enumerate(nf):
        s = _ClipState(idx=i, content_frames=max(0, n - 1), all_tokens=list(init_tokens), lang_token=lang_token)
        s.result.duration = len(pcm_list[i]) / 16000.0
        s.done = s.content_frames <= 0
        states.append(s)
    max_init = int(round(opts.max_initial_timestamp / TIME_PRECISION))
    sampling = opts.temperature > 0
    beam = 1 if sampling else max(1, int(opts.beam_size))
    group = max(1, int(opts.best_of)) if sampling else beam  # decoder rows per window
    B = max(1, min(engine.max_batch, getattr(engine, "max_rows", engine.max_batch) // group))
    calls = 0
    while True:
        active = [s for s in states if not s.done]
        if not active:
            break
        # group due windows by prompt (prefix) length and by "language known"
        groups: dict = {}
        for s in active:
            prev = s.all_tokens[s.prompt_reset_since:]
            prefix = ([st.sot_prev] + prev[-(448 // 2 - 1):]) if prev else []
            groups.setdefault((len(prefix), s.lang_token is None), []).append((s, prefix))
        for (_plen, _detect), members in groups.items():
            for lo in range(0, len(members), B):
                chunk = members[lo:lo + B]
                wins = []
                for s, _ in chunk:
                    size = min(N_FRAMES, s.content_frames - s.seek)
                    wins.append((s.idx, s.seek, size))
                engine.encode(wins)
                langs = None if _detect else [s.lang_token for s, _ in chunk]
                max_length = 448
                if opts.max_new_tokens is not None:
                    max_length = _plen + 3 + (1 if opts.without_timestamps else 0) + int(opts.max_new_tokens)
                    if max_length > 448:
                        raise ValueError(f"the prompt is {max_length - int(opts.max_new_tokens)} tokens and "
                                         f"max_new_tokens is {opts.max_new_tokens}: their sum exceeds the "
                                         "model's maximum length (448)")
                cfg = DecodeConfig(max_length=max_length, task=opts.task, language_token=None, suppress_tokens=suppress,
                                   suppress_blank=opts.suppress_blank, without_timestamps=opts.without_timestamps,
                                   max_initial_timestamp_index=max_init, beam_size=beam, patience=opts.patience,
                                   length_penalty=opts.length_penalty, temperature=opts.temperature,
                                   best_of=opts.best_of, seed=(opts.seed + 0x9E3779B1 * calls) & (2**64 - 1))
                if opts.tokens_per_second:
                    cfg.token_budget = tuple(int(np.ceil(opts.tokens_per_second * z * FRAME_SEC)) + 2
                                             for _, _, z in wins)
                calls += 1
                prefixes = [p for _, p in chunk] if _plen else None
                outs = engine.decode(len(chunk), cfg, prefix=prefixes, languages=langs)
                for (s, _), w, out in zip(chunk, wins, outs):
                    _consume(s, w, out, opts, tok)
    for s in states:
        code = tok.language_code(s.lang_token) if s.lang_token is not None else (opts.language or "en")
        s.result.language = code
    return [s.result for s in states]


# ------------------------------------------------------------ one clip at a time
# (the runner's decode-session lanes, runner.py: each clip's seek loop advances on its own,
# its next window queued into the session as soon as the previous one is consumed)

def session_supported(opts: TranscribeOptions) -> bool:
    """Decode sessions (osw_session_*) hold one decode configuration for every window:
    temperature 0, beam_size <= 5, and no max_new_tokens (whose max_length depends on
    each window's prompt length)."""
    return not (opts.temperature > 0) and opts.max_new_tokens is None and 1 <= int(opts.beam_size) <= 5


def session_config(opts: TranscribeOptions, suppress: tuple) -> DecodeConfig:
    """The session-wide decode configuration (transcribe_clips' per-call one, minus the
    per-window prefix, language and token budget)."""
    return DecodeConfig(max_length=448, task=opts.task, language_token=None, suppress_tokens=suppress,
                        suppress_blank=opts.suppress_blank, without_timestamps=opts.without_timestamps,
                        max_initial_timestamp_index=int(round(opts.max_initial_timestamp / TIME_PRECISION)),
                        beam_size=max(1, int(opts.beam_size)), patience=opts.patience,
                        length_penalty=opts.length_penalty)


def clip_state(idx: int, pcm: np.ndarray, opts: TranscribeOptions, tok: WhisperTokenizer) -> _ClipState:
    """transcribe_clips' per-clip state (log_mel's frame count is len // 160 + 1, the
    content frames one fewer)."""
    lang_token = tok.language_token(opts.language) if (opts.language and opts.task == "transcribe") else None
    init_tokens = tok.encode(" " + opts.initial_prompt.strip()) if opts.initial_prompt else []
    s = _ClipState(idx=idx, content_frames=len(pcm) // HOP_LENGTH, all_tokens=list(init_tokens),
                   lang_token=lang_token)
    s.result.duration = len(pcm) / 16000.0
    s.done = s.content_frames <= 0
    return s


def next_window(s: _ClipState, opts: TranscribeOptions, tok: WhisperTokenizer) -> dict:
    """The clip's next window: seek, segment_size, prompt prefix, language, token budget."""
    prev = s.all_tokens[s.prompt_reset_since:]
    prefix = ([tok.special.sot_prev] + prev[-(448 // 2 - 1):]) if prev else []
    size = min(N_FRAMES, s.content_frames - s.seek)
    budget = int(np.ceil(opts.tokens_per_second * size * FRAME_SEC)) + 2 if opts.tokens_per_second else 0
    return dict(seek=s.seek, segment_size=size, prefix=prefix, language_token=s.lang_token, token_budget=budget)


def consume_window(s: _ClipState, win: dict, out, opts: TranscribeOptions, tok: WhisperTokenizer) -> None:
    _consume(s, (s.idx, win["seek"], win["segment_size"]), out, opts, tok)


def finish_clip(s: _ClipState, opts: TranscribeOptions, tok: WhisperTokenizer) -> ClipResult:
    s.result.language = tok.language_code(s.lang_token) if s.lang_token is not None else (opts.language or "en")
    return s.result


def _consume(s: _ClipState, win, out, opts: TranscribeOptions, tok: WhisperTokenizer) -> None:
    st = tok.special
    _, seek, segment_size = win
    if s.lang_token is None:
        s.lang_token = out.language
    tokens = out.tokens
    avg_logprob = out.sum_logprob / (len(tokens) + 1)
    text = tok.decode(tokens).strip()
    cr = compression_ratio(text)
    if opts.no_speech_threshold is not None:
        skip = out.no_speech_prob > opts.no_speech_threshold
        if opts.log_prob_threshold is not None and avg_logprob > opts.log_prob_threshold:
            skip = False
        if skip:
            s.seek = seek + segment_size
            s.done = s.seek >= s.content_frames
            return
    time_offset = seek * FRAME_SEC
    segs, new_seek, _ = split_segments_by_timestamps(tokens, st.timestamp_begin, time_offset, segment_size,
                                                     segment_size * FRAME_SEC, seek)
    for sg in segs:
        t = sg["tokens"]
        txt = tok.decode(t)
        if sg["start"] == sg["end"] or not txt.strip():
            continue
        s.all_tokens.extend(t)
        s.result.segments.append(Segment(id=len(s.result.segments), seek=seek, start=sg["start"], end=sg["end"],
                                         text=txt, tokens=list(t), temperature=opts.temperature,
                                         avg_logprob=avg_logprob, compression_ratio=cr,
                                         no_speech_prob=out.no_speech_prob))
    if not opts.condition_on_previous_text or opts.temperature > opts.prompt_reset_on_temperature:
        s.prompt_reset_since = len(s.all_tokens)
    s.seek = new_seek
    s.done = s.seek >= s.content_frames


def verbose_dict(task: str, res: ClipResult) -> dict:
    """The ``verbose_json`` shape of ``src/backends/faster_whisper.py:251-272``."""
    full = "".join(sg.text for sg in res.segments).strip()
    return {
        "task": task, "language": res.language, "duration": res.duration, "text": full,
        "segments": [{"id": i, "seek": int(sg.seek), "start": sg.start, "end": sg.end, "text": sg.text,
                      "tokens": list(sg.tokens) if sg.tokens else [], "temperature": sg.temperature,
                      "avg_logprob": sg.avg_logprob, "compression_ratio": sg.compression_ratio,
                      "no_speech_prob": sg.no_speech_prob} for i, sg in enumerate(res.segments)],
    }


def _ts(seconds: float, sep: str) -> str:
    h = int(seconds // 3600)
    m = int((seconds % 3600) // 60)
    s = int(seconds % 60)
    ms = int((seconds % 1) * 1000)
    return f"{h:02d}:{m:02d}:{s:02d}{sep}{ms:03d}"


def to_srt(segments) -> str:
    """``FasterWhisperBackend._to_srt`` (src/backends/faster_whisper.py:313-321)."""
    return "\n".join(f"{i}\n{_ts(s.start, ',')} --> {_ts(s.end, ',')}\n{s.text.strip()}\n"
                     for i, s in enumerate(segments, 1))


def to_vtt(segments) -> str:
    """``FasterWhisperBackend._to_vtt`` (src/backends/faster_whisper.py:323-330)."""
    lines = ["WEBVTT\n"]
    for s in segments:
        lines.append(f"{_ts(s.start, '.')} --> {_ts(s.end, '.')}\n{s.text.strip()}\n")
    return "\n".join(lines)


def shape_response(task: str, res: ClipResult, response_format: str) -> dict:
    """Return shapes by format (src/backends/faster_whisper.py:251-281)."""
    full = "".join(sg.text for sg in res.segments).strip()
    if response_format == "verbose_json":
        return verbose_dict(task, res)
    if response_format == "text":
        return {"text": full, "raw_text": True}
    if response_format == "srt":
        return {"text": to_srt(res.segments), "raw_text": True}
    if response_format == "vtt":
        return {"text": to_vtt(res.segments), "raw_text": True}
    return {"text": full}


def np_int16(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.int16)
