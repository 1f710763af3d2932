"""ORACLE (test infrastructure only) — faster-whisper's long-form seek loop.

Restates faster-whisper 1.2.1 ``WhisperModel.generate_segments`` (upstream
``faster_whisper/transcribe.py``, not vendored) for one file at temperature 0 with a
scalar temperature (the reference passes ``temperature`` as a scalar,
``src/backends/faster_whisper.py:238``, so there is no fallback):

* the log-mel is computed once for the whole file; ``content_frames = n_frames - 1``;
  each window is ``mel[:, seek:seek + segment_size]`` padded to 3000 frames with
  ``segment_size = min(3000, content_frames - seek)``;
* the prompt is ``[<|startofprev|>] + previous_tokens[-(448 // 2 - 1):]`` when
  ``condition_on_previous_text`` and earlier windows produced text, then
  ``[<|startoftranscript|>, language, task]``;
* a window is skipped (``seek += segment_size``) when ``no_speech_prob >
  no_speech_threshold`` and ``avg_logprob = sum_logprob / (len(tokens) + 1)`` is not
  above ``log_prob_threshold``;
* otherwise its tokens are split at consecutive timestamp pairs
  (``_split_segments_by_timestamps``): a single timestamp ending moves the seek by
  the whole window, else by twice the last timestamp's position (2 mel frames per
  timestamp step of 0.02 s); segments with start == end or blank text are dropped
  and do not enter the previous-text prompt.

The decoder is injected (``decode_window``), so the GPU's own encoder outputs can be
decoded by the oracle window by window (tests/test_gpu_longform.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

N_FRAMES = 3000
TIME_PRECISION = 0.02
INPUT_STRIDE = 2
FRAME_SEC = 0.01


@dataclass
class SeekOptions:
    condition_on_previous_text: bool = True
    no_speech_threshold: float | None = 0.6
    log_prob_threshold: float | None = -1.0


@dataclass
class Window:
    seek: int
    size: int
    prompt: list
    tokens: list
    skipped: bool = False
    segments: list = field(default_factory=list)   # (start, end, tokens)


def split_by_timestamps(tokens, tb, time_offset, segment_size, segment_duration, seek):
    """faster-whisper ``_split_segments_by_timestamps`` (returns segments, next seek)."""
    segs = []
    single_ending = len(tokens) >= 2 and tokens[-2] < tb <= tokens[-1]
    cons = [i for i in range(1, len(tokens)) if tokens[i] >= tb and tokens[i - 1] >= tb]
    if cons:
        slices = cons + ([len(tokens)] if single_ending else [])
        last = 0
        for cur in slices:
            part = tokens[last:cur]
            segs.append((time_offset + (part[0] - tb) * TIME_PRECISION,
                         time_offset + (part[-1] - tb) * TIME_PRECISION, part))
            last = cur
        if single_ending:
            seek += segment_size
        else:
            seek += (tokens[last - 1] - tb) * INPUT_STRIDE
    else:
        duration = segment_duration
        ts = [t for t in tokens if t >= tb]
        if ts and ts[-1] != tb:
            duration = (ts[-1] - tb) * TIME_PRECISION
        segs.append((time_offset, time_offset + duration, tokens))
        seek += segment_size
    return segs, seek


def seek_loop(decode_window, n_frames: int, st, decode_text, opts: SeekOptions = SeekOptions(),
              initial_tokens=()):
    """decode_window(seek, size, prev_tokens) -> (tokens, sum_logprob, no_speech_prob);
    decode_text(tokens) -> str; initial_tokens: the encoded initial prompt
    (``tokenizer.encode(" " + initial_prompt.strip())``), the first previous text.
    Returns the list of Windows in order."""
    content = max(0, n_frames - 1)
    seek, all_tokens, reset_since, out = 0, list(initial_tokens), 0, []
    while seek < content:
        size = min(N_FRAMES, content - seek)
        prev = all_tokens[reset_since:]
        prompt = ([st.sot_prev] + prev[-(448 // 2 - 1):]) if prev else []
        tokens, sum_lp, nsp = decode_window(seek, size, prompt)
        w = Window(seek, size, prompt, list(tokens))
        out.append(w)
        avg = sum_lp / (len(tokens) + 1)
        if opts.no_speech_threshold is not None and nsp > opts.no_speech_threshold and not (
                opts.log_prob_threshold is not None and avg > opts.log_prob_threshold):
            w.skipped = True
            seek += size
            continue
        segs, new_seek = split_by_timestamps(list(tokens), st.timestamp_begin, seek * FRAME_SEC, size,
                                             size * FRAME_SEC, seek)
        for a, b, t in segs:
            if a == b or not decode_text(t).strip():
                continue
            all_tokens.extend(t)
            w.segments.append((a, b, list(t)))
        if not opts.condition_on_previous_text:
            reset_since = len(all_tokens)
        seek = new_seek
    return out
