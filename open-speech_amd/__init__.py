"""open_speech_amd — MI355X-native Whisper transcription backend for open-speech.

Drop-in for the reference's STT plugin seam (``src/backends/base.py:10-38``): the
host side here mirrors ``FasterWhisperBackend`` (``src/backends/faster_whisper.py``)
and calls the C-ABI library ``libosw_hip.so`` (declared in ``include/osw.h``) whose
hot path is hand-written HIP for gfx950.
"""
from .dims import LARGE_V3_TURBO, MICRO_TEST, TINY_TEST, WhisperDims  # noqa: F401

__all__ = ["WhisperDims", "LARGE_V3_TURBO", "TINY_TEST", "MICRO_TEST"]
