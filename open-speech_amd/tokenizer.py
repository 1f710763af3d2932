"""Tokenizer-side helpers: suppressed-token sets and token → text decoding.

Mirrors faster-whisper 1.2.1 ``get_suppressed_tokens`` and ``Tokenizer`` (upstream,
not vendored).  ``suppress_tokens=[-1]`` expands to the tokenizer's
``non_speech_tokens`` plus ``[transcribe, translate, sot, sot_prev, sot_lm]``.

When a model directory provides ``tokenizer.json`` the non-speech set is computed
from it exactly as upstream does (symbols and their space-prefixed forms encoded
to single tokens).  Without one, the multilingual Whisper table below is used —
it is the text-token part of the published ``suppress_tokens`` list of the
multilingual checkpoints' generation config (parity unpinned: there is no
tokenizer in this image to recompute it).
"""
from __future__ import annotations

import os
import zlib

from .dims import LANGUAGE_CODES, SpecialTokens

NON_SPEECH_TOKENS_MULTILINGUAL = (
    1, 2, 7, 8, 9, 10, 14, 25, 26, 27, 28, 29, 31, 58, 59, 60, 61, 62, 63, 90, 91, 92, 93, 359,
    503, 522, 542, 873, 893, 902, 918, 922, 931, 1350, 1853, 1982, 2460, 2627, 3246, 3253, 3268,
    3536, 3846, 3961, 4183, 4667, 6585, 6647, 7273, 9061, 9383, 10428, 10929, 11938, 12033, 12331,
    12562, 13793, 14157, 14635, 15265, 15618, 16553, 16604, 18362, 18956, 20075, 21675, 22520,
    26130, 26161, 26435, 28279, 29464, 31650, 32302, 32470, 36865, 42863, 47425, 49870, 50254,
)

_SYMBOLS = list('"#()*+/:;<=>@[\\]^_`{|}~「」『』')
_SYMBOLS += "<< >> <<< >>> -- --- -( -[ (' (\" (( )) ((( ))) [[ ]] {{ }} ♪♪ ♪♪♪".split()
_MISC = set("♩♪♫♬♭♮♯")


class WhisperTokenizer:
    """Thin wrapper; text decoding needs a ``tokenizer.json`` (``tokenizers`` package)."""

    def __init__(self, n_vocab: int, tokenizer_json: str | None = None):
        self.special = SpecialTokens.for_vocab(n_vocab)
        self.n_vocab = n_vocab
        self._tok = None
        if tokenizer_json and os.path.exists(tokenizer_json):
            from tokenizers import Tokenizer  # available in the image

            self._tok = Tokenizer.from_file(tokenizer_json)

    @property
    def has_text(self) -> bool:
        return self._tok is not None

    def encode(self, text: str) -> list[int]:
        if self._tok is None:
            return []
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, tokens) -> str:
        text_tokens = [int(t) for t in tokens if int(t) < self.special.eot]
        if self._tok is None:
            return "".join(f"<|{t}|>" for t in text_tokens)
        return self._tok.decode(text_tokens, skip_special_tokens=False)

    def non_speech_tokens(self) -> tuple:
        if self._tok is None:
            return NON_SPEECH_TOKENS_MULTILINGUAL
        result = {self.encode(" -")[0], self.encode(" '")[0]}
        for symbol in _SYMBOLS + list(_MISC):
            for tokens in (self.encode(symbol), self.encode(" " + symbol)):
                if len(tokens) == 1 or symbol in _MISC:
                    result.add(tokens[0])
        return tuple(sorted(result))

    def language_code(self, lang_token: int) -> str:
        i = lang_token - self.special.first_lang
        return LANGUAGE_CODES[i] if 0 <= i < len(LANGUAGE_CODES) else "en"

    def language_token(self, code: str) -> int:
        try:
            i = LANGUAGE_CODES.index(code)
        except ValueError as e:
            raise ValueError(f"unsupported language: {code!r}") from e
        if i >= self.special.n_langs:
            raise ValueError(f"language {code!r} not in this vocabulary")
        return self.special.first_lang + i


def get_suppressed_tokens(tok: WhisperTokenizer, suppress_tokens=(-1,)) -> tuple:
    st = tok.special
    s = list(suppress_tokens or [])
    if -1 in s:
        s = [t for t in s if t >= 0]
        s.extend(tok.non_speech_tokens())
    s.extend([st.transcribe, st.translate, st.sot, st.sot_prev, st.sot_lm])
    return tuple(sorted(set(s)))


def compression_ratio(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b)) if b else 0.0
