"""ctypes binding of libosw_hip.so (include/osw.h).

The product path has NO CPU fallback: if the library is missing or the device is
absent, loading raises ``RuntimeError`` with the reason.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OSW_LIB", os.path.join(_HERE, "lib", "libosw_hip.so"))

OSW_OK = 0


class osw_dims(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_mels", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                                          "n_vocab", "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer")]


class osw_window(C.Structure):
    _fields_ = [("clip", C.c_int32), ("seek", C.c_int32), ("segment_size", C.c_int32)]


class osw_decode_opts(C.Structure):
    _fields_ = [("task_token", C.c_int32), ("language_token", C.c_int32), ("suppress_blank", C.c_int32),
                ("without_timestamps", C.c_int32), ("max_initial_timestamp_index", C.c_int32),
                ("max_length", C.c_int32), ("suppress_tokens", C.POINTER(C.c_int32)), ("n_suppress", C.c_int32),
                ("eot", C.c_int32), ("sot", C.c_int32), ("sot_prev", C.c_int32), ("no_speech", C.c_int32),
                ("no_timestamps", C.c_int32), ("timestamp_begin", C.c_int32), ("blank", C.c_int32),
                ("first_lang", C.c_int32), ("n_langs", C.c_int32),
                ("prefix_tokens", C.POINTER(C.c_int32)), ("n_prefix", C.c_int32),
                ("language_tokens", C.POINTER(C.c_int32)),
                ("beam_size", C.c_int32), ("patience", C.c_float), ("length_penalty", C.c_float),
                ("num_hypotheses", C.c_int32), ("temperature", C.c_float), ("best_of", C.c_int32),
                ("seed", C.c_uint64), ("token_budget", C.POINTER(C.c_int32))]


class osw_window_result(C.Structure):
    _fields_ = [("tokens", C.POINTER(C.c_int32)), ("max_tokens", C.c_int32), ("n_tokens", C.POINTER(C.c_int32)),
                ("sum_logprob", C.POINTER(C.c_float)), ("no_speech_prob", C.POINTER(C.c_float)),
                ("language", C.POINTER(C.c_int32)), ("logits_dump", C.POINTER(C.c_float)),
                ("dump_steps", C.c_int32)]


class osw_session_window(C.Structure):
    _fields_ = [("tag", C.c_int64), ("seek", C.c_int32), ("segment_size", C.c_int32), ("language_token", C.c_int32),
                ("token_budget", C.c_int32), ("n_prefix", C.c_int32), ("prefix", C.POINTER(C.c_int32)),
                ("clip", C.c_int64)]


class osw_profile(C.Structure):
    _fields_ = [("mel_ms", C.c_double), ("encoder_ms", C.c_double), ("crosskv_ms", C.c_double),
                ("decoder_ms", C.c_double), ("total_ms", C.c_double), ("decode_steps", C.c_int64),
                ("enc_gemm_ms", C.c_double), ("enc_gemm_launches", C.c_int64), ("enc_gemm_flops", C.c_double),
                ("enc_attn_ms", C.c_double), ("enc_attn_launches", C.c_int64), ("enc_attn_flops", C.c_double),
                ("mel_kernel_ms", C.c_double), ("mel_kernel_launches", C.c_int64), ("mel_kernel_bytes", C.c_double),
                ("xattn_ms", C.c_double), ("xattn_launches", C.c_int64), ("xattn_bytes", C.c_double)]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


P = C.POINTER
_SIGS = {
    "osw_version": (C.c_char_p, []),
    "osw_last_error": (C.c_char_p, []),
    "osw_device_count": (C.c_int, [P(C.c_int32)]),
    "osw_create": (C.c_int, [P(osw_dims), C.c_int32, C.c_int32, P(C.c_void_p)]),
    "osw_destroy": (C.c_int, [C.c_void_p]),
    "osw_create_sibling": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_void_p)]),
    "osw_set_weight": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int64]),
    "osw_get_weight": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int64]),
    "osw_init_weight_uniform": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_int64, C.c_float, C.c_float,
                                          C.c_int64, C.c_int64]),
    "osw_finalize": (C.c_int, [C.c_void_p]),
    "osw_log_mel": (C.c_int, [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int32, C.c_int32, P(C.c_int32)]),
    "osw_get_mel": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_float), C.c_int64]),
    "osw_encode_windows": (C.c_int, [C.c_void_p, P(osw_window), C.c_int32]),
    "osw_get_encoder_output": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_float), C.c_int64]),
    "osw_decode_windows": (C.c_int, [C.c_void_p, C.c_int32, P(osw_decode_opts), P(osw_window_result)]),
    "osw_transcribe_batch": (C.c_int, [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int32, C.c_int32,
                                       P(osw_decode_opts), P(osw_window_result)]),
    "osw_transcribe_refill": (C.c_int, [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int32, C.c_int32,
                                        P(osw_decode_opts), P(osw_window_result), C.c_int32]),
    "osw_session_begin": (C.c_int, [C.c_void_p, P(osw_decode_opts)]),
    "osw_session_add": (C.c_int, [C.c_void_p, C.c_void_p, P(C.c_int64), C.c_int32, P(osw_session_window)]),
    "osw_session_step": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, P(osw_window_result), P(C.c_int64), C.c_int32,
                                   P(C.c_int32), P(C.c_int32), P(C.c_int32)]),
    "osw_session_release_clip": (C.c_int, [C.c_void_p, C.c_int64]),
    "osw_session_end": (C.c_int, [C.c_void_p]),
    "osw_encoder_layer_debug": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_float), P(C.c_float), C.c_int32]),
    "osw_debug_gemm": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                                 P(C.c_float), C.c_int32, P(C.c_float)]),
    "osw_debug_hold_capture": (C.c_int, [C.c_void_p, C.c_int32]),
    "osw_set_encoder_baton_min": (C.c_int, [C.c_void_p, C.c_int32]),
    "osw_set_profiling": (C.c_int, [C.c_void_p, C.c_int32]),
    "osw_get_profile": (C.c_int, [C.c_void_p, P(osw_profile)]),
    "osw_stream": (C.c_void_p, [C.c_void_p]),
    "osw_ingest_mean_square": (C.c_int, [C.c_int32, P(C.c_int16), C.c_int64, C.c_int32, P(C.c_float)]),
    "osw_ingest_apply_gain": (C.c_int, [C.c_int32, P(C.c_int16), C.c_int64, C.c_int32, C.c_int32, C.c_float,
                                        P(C.c_int16)]),
    "osw_ingest_resample": (C.c_int, [C.c_int32, P(C.c_int16), C.c_int64, C.c_int32, C.c_int32, P(C.c_float),
                                      C.c_int32, P(C.c_int16), C.c_int64]),
}
EXPORTED = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


def load() -> C.CDLL:
    """Load libosw_hip.so (raises RuntimeError if it is absent: no fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libosw_hip.so not found at {LIB_PATH}: build it with `python __graft_entry__.py` "
                               "or `make -C open-speech_amd/csrc` (there is no CPU fallback)")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


OSW_EHIP = -100
OSW_ECAPTURE = -102


class OswError(RuntimeError):
    """A non-zero return code of libosw_hip.so (``rc``) with its osw_last_error() text."""

    def __init__(self, msg: str, rc: int):
        super().__init__(msg)
        self.rc = rc


class OswDeviceError(OswError):
    """OSW_EHIP: a HIP runtime error on the context's device (the batcher fails the GPU over)."""


class OswCaptureError(OswError):
    """OSW_ECAPTURE: a stream capture was refused or invalidated.  Not a device fault: the
    context and the GPU stay usable (the batcher fails only the affected requests)."""


def check(rc: int, what: str = "") -> None:
    if rc != OSW_OK:
        msg = load().osw_last_error().decode(errors="replace")
        cls = {OSW_EHIP: OswDeviceError, OSW_ECAPTURE: OswCaptureError}.get(rc, OswError)
        raise cls(f"{what} failed ({rc}): {msg}", rc)
