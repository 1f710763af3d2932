"""Whisper model dimensions and special-token ids.

The reference never sees these numbers directly: they live inside the CTranslate2
model it loads at ``src/backends/faster_whisper.py:40-45`` (default model id
``deepdml/faster-whisper-large-v3-turbo-ct2``, ``src/config.py:141``).  They are
the published Whisper architecture constants.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

SAMPLE_RATE = 16000
N_FFT = 400
HOP_LENGTH = 160
CHUNK_LENGTH = 30
N_SAMPLES = CHUNK_LENGTH * SAMPLE_RATE      # 480000 samples per 30 s window
N_FRAMES = N_SAMPLES // HOP_LENGTH          # 3000 mel frames per window
TIME_PRECISION = 0.02                       # seconds per timestamp token
INPUT_STRIDE = 2                            # mel frames per encoder position


@dataclass(frozen=True)
class WhisperDims:
    n_mels: int = 128
    n_audio_ctx: int = 1500
    n_audio_state: int = 1280
    n_audio_head: int = 20
    n_audio_layer: int = 32
    n_vocab: int = 51866
    n_text_ctx: int = 448
    n_text_state: int = 1280
    n_text_head: int = 20
    n_text_layer: int = 4

    @property
    def head_dim(self) -> int:
        return self.n_audio_state // self.n_audio_head

    def as_dict(self) -> dict:
        return asdict(self)


# whisper-large-v3-turbo (808,878,080 params)
LARGE_V3_TURBO = WhisperDims()
# reduced "tiny-like" dims used by the golden fixtures
TINY_TEST = WhisperDims(n_mels=80, n_audio_state=384, n_audio_head=6, n_audio_layer=4,
                        n_text_state=384, n_text_head=6, n_text_layer=4)
# very small dims for fast CPU tests (still real vocab/contexts)
MICRO_TEST = WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                         n_text_state=128, n_text_head=2, n_text_layer=2)

PRESETS = {
    "large-v3-turbo": LARGE_V3_TURBO,
    "tiny-test": TINY_TEST,
    "micro-test": MICRO_TEST,
}


@dataclass(frozen=True)
class SpecialTokens:
    """Special token ids of the multilingual Whisper vocabulary.

    For n_vocab == 51866 (large-v3 / turbo) the language block has 100 entries
    (``<|yue|>`` added), shifting every id after it by one relative to v2.
    """
    eot: int
    sot: int
    first_lang: int
    n_langs: int
    translate: int
    transcribe: int
    sot_lm: int
    sot_prev: int
    no_speech: int
    no_timestamps: int
    timestamp_begin: int
    blank: int = 220  # tokenizer.encode(" ") for the GPT-2 derived BPE

    @classmethod
    def for_vocab(cls, n_vocab: int) -> "SpecialTokens":
        n_langs = 100 if n_vocab >= 51866 else 99
        first_lang = 50259
        after = first_lang + n_langs
        return cls(eot=50257, sot=50258, first_lang=first_lang, n_langs=n_langs,
                   translate=after, transcribe=after + 1, sot_lm=after + 2,
                   sot_prev=after + 3, no_speech=after + 4, no_timestamps=after + 5,
                   timestamp_begin=after + 6)


# Language codes in token order (openai-whisper tokenizer.LANGUAGES order).
LANGUAGE_CODES = (
    "en zh de es ru ko fr ja pt tr pl ca nl ar sv it id hi fi vi he uk el ms cs ro da hu ta no "
    "th ur hr bg lt la mi ml cy sk te fa lv bn sr az sl kn et mk br eu is hy ne mn bs kk sq sw "
    "gl mr pa si km sn yo so af oc ka be tg sd gu am yi lo uz fo ht ps tk nn mt sa lb my bo tl "
    "mg as tt haw ln ha ba jw su yue"
).split()
