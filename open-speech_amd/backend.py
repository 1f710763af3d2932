"""``HipWhisperBackend`` — the drop-in for ``FasterWhisperBackend``
(``src/backends/faster_whisper.py:19-310``), satisfying the ``STTBackend`` Protocol
(``src/backends/base.py:10-38``).

Registration without editing ``router.py``: ``install(router)``
puts the backend under the key ``"faster-whisper"`` — the provider key
``ModelManager`` resolves every STT id to (``src/model_manager.py:20-28,116-126``) —
and makes it the router's ``_default_backend`` (``src/router.py:23-31``), the same
seam the reference's own tests patch (``tests/test_api.py:25-26``).

Kept exactly: ``_models`` / ``_loaded_at`` / ``_last_used`` dicts (read by
``src/lifecycle.py:46-73``), idempotent ``load_model``, auto-load on first use,
``_last_used`` refresh per call, return shapes per ``response_format``, exceptions
propagated to the caller (HTTP 500 / WS error / Wyoming "").
Decoding is beam search width 5 like the reference (``STT_HIP_BEAM_SIZE=1`` selects
greedy, the parity mode).  Differences by design: audio bytes are parsed in memory
(no temp file, no PyAV) and concurrent calls are batched on the GPU behind the
blocking ``transcribe``.
"""
from __future__ import annotations

import gc
import logging
import os
import shutil
import threading
import time
from pathlib import Path
from typing import Any

from . import model_store
from .audio import decode_audio_bytes
from .runner import BatchRunner
from .segments import TranscribeOptions, shape_response
from .tokenizer import WhisperTokenizer

logger = logging.getLogger(__name__)


class _Settings:
    """Reads ``src.config.settings`` when running inside open-speech, else the same
    env vars (``src/config.py:141-145``) plus this backend's own knobs."""

    def __init__(self):
        try:
            from src.config import settings as s  # type: ignore
        except Exception:
            s = None
        self._s = s

    def get(self, name: str, default=None):
        if self._s is not None and hasattr(self._s, name):
            return getattr(self._s, name)
        v = os.environ.get(name.upper())
        if v is None:
            return default
        if isinstance(default, bool):
            return v.lower() in ("1", "true", "yes")
        if isinstance(default, int):
            return int(v)
        return v


def _loaded_model_info(**kw):
    try:
        from src.models import LoadedModelInfo  # type: ignore

        return LoadedModelInfo(**kw)
    except Exception:
        return dict(kw)


class _Model:
    def __init__(self, src, runner, tokenizer, engines):
        self.src, self.runner, self.tokenizer, self.engines = src, runner, tokenizer, engines


class HipWhisperBackend:
    """STT backend running Whisper on MI355X GPUs through libosw_hip.so."""

    name = "faster-whisper"

    def __init__(self, engine_factory=None, length_control: float | None = None) -> None:
        """``length_control`` (benchmarks only, not a reference option): end every window
        after this many tokens per second of audio, since random weights never emit
        <|endoftext|> (segments.TranscribeOptions.tokens_per_second)."""
        self._length_control = length_control
        self._models: dict[str, Any] = {}
        self._loaded_at: dict[str, float] = {}
        self._last_used: dict[str, float] = {}
        self._load_lock = threading.Lock()
        self._settings = _Settings()
        self._engine_factory = engine_factory

    # ------------------------------------------------------------ config
    @property
    def device_label(self) -> str:
        return f"rocm:{','.join(str(g) for g in self._gpu_ids())}"

    def _gpu_ids(self) -> list[int]:
        spec = os.environ.get("STT_HIP_GPUS", "0")
        if spec == "all":
            from . import _lib
            import ctypes as C

            n = C.c_int32()
            _lib.check(_lib.load().osw_device_count(C.byref(n)), "osw_device_count")
            return list(range(n.value))
        return [int(x) for x in spec.split(",") if x.strip()]

    # ------------------------------------------------------------ lifecycle
    def load_model(self, model_id: str) -> None:
        with self._load_lock:
            if model_id in self._models:
                logger.info("Model %s already loaded", model_id)
                return
            src = model_store.resolve(model_id, self._settings.get("stt_model_dir", None))
            max_batch = int(os.environ.get("STT_HIP_MAX_BATCH", "16"))
            wait_ms = float(os.environ.get("STT_HIP_BATCH_WAIT_MS", "5"))
            gap_ms = float(os.environ.get("STT_HIP_BATCH_GAP_MS", "1"))
            factory = self._engine_factory or _default_engine_factory
            engines = []
            try:
                weights = model_store.load_weights(src)
                for gpu in self._gpu_ids():
                    eng = factory(src.dims, gpu, max_batch)
                    if weights is not None:
                        eng.load_weights(weights)
                    else:
                        eng.init_random(seed=src.seed)
                    engines.append(eng)
                    # extra lanes on the same GPU share the weights: one batch's encoder
                    # (MFMA-bound) overlaps another's decoder (HBM/latency-bound)
                    for _ in range(max(1, int(os.environ.get("STT_HIP_LANES", "3"))) - 1):
                        if hasattr(eng, "sibling"):
                            engines.append(eng.sibling())
            except Exception:
                for e in engines:
                    e.close()
                raise
            # pipelined lanes (runner.py): the lanes of a GPU take turns on the encoder, so
            # one batch encodes while the others decode
            split = os.environ.get("STT_HIP_SPLIT", "1") != "0"
            # continuous batching (runner._SessionLane): every lane drives a decode session,
            # windows of any request admitted between chunks of decoder steps.  Mixed-length
            # REST load (tools/rest_probe.py mix, 16 callers): 52.8 -> 67.3 calls/s, p50
            # 236 -> 148 ms; config 5 within noise of batch-at-a-time (165.7 / 169.0 calls/s,
            # gpurun_out/r05_s3, r05_s4).  STT_HIP_CONTINUOUS=0: batch at a time.
            continuous = os.environ.get("STT_HIP_CONTINUOUS", "1") != "0"
            spread = os.environ.get("STT_HIP_SPREAD_MS")
            tok = WhisperTokenizer(src.dims.n_vocab, src.tokenizer_json)
            runner = BatchRunner(engines, tok, max_wait_ms=wait_ms, gap_ms=gap_ms, split=split,
                                 continuous=continuous, refill_min=int(os.environ.get("STT_HIP_REFILL_MIN", "1")),
                                 spread_ms=float(spread) if spread else None)
            self._models[model_id] = _Model(src, runner, tok, engines)
            now = time.time()
            self._loaded_at[model_id] = now
            self._last_used[model_id] = now
            logger.info("Model %s loaded on %s", model_id, self.device_label)

    def unload_model(self, model_id: str) -> None:
        m = self._models.pop(model_id, None)
        if m is None:
            return
        self._loaded_at.pop(model_id, None)
        self._last_used.pop(model_id, None)
        m.runner.close()
        gc.collect()
        logger.info("Model %s unloaded", model_id)

    def loaded_models(self) -> list:
        now = time.time()
        ttl = int(self._settings.get("stt_model_ttl", 300) or 0)
        default_model = self._settings.get("stt_default_model", self._settings.get("stt_model", None))
        return [
            _loaded_model_info(
                model=mid, backend=self.name, device=self.device_label, compute_type="float16",
                loaded_at=self._loaded_at[mid], last_used_at=self._last_used.get(mid),
                is_default=(mid == default_model),
                ttl_remaining=(None if (mid == default_model or ttl == 0)
                               else max(0.0, ttl - (now - self._last_used.get(mid, now)))))
            for mid in list(self._models)
        ]

    def is_model_loaded(self, model_id: str) -> bool:
        return model_id in self._models

    # ------------------------------------------------------------ cache (duck-typed by the router)
    def _cache_root(self) -> Path:
        return Path(model_store.cache_dirs(self._settings.get("stt_model_dir", None))[0])

    def list_cached_models(self) -> list[dict[str, Any]]:
        """``FasterWhisperBackend.list_cached_models`` (src/backends/faster_whisper.py:103-172):
        with ``STT_MODEL_DIR`` set, every non-hidden directory counts (``models--Org--Name``
        as ``Org/Name``, anything else under its own name); in the HF cache only
        ``models--Org--Name``."""
        root = self._cache_root()
        custom = bool(self._settings.get("stt_model_dir", None))
        out, seen = [], set()
        default_model = self._settings.get("stt_default_model", None)
        if root.exists():
            for p in root.iterdir():
                if not p.is_dir() or (custom and p.name.startswith(".")):
                    continue
                if p.name.startswith("models--"):
                    parts = p.name.split("--", 2)
                    if len(parts) != 3:
                        if not custom:
                            continue
                        mid = p.name
                    else:
                        mid = f"{parts[1]}/{parts[2]}"
                elif custom:
                    mid = p.name
                else:
                    continue
                seen.add(mid)
                size = sum(f.stat().st_size for f in p.rglob("*") if f.is_file()) / (1024 * 1024)
                out.append({"model": mid, "loaded": mid in self._models, "is_default": mid == default_model,
                            "size_mb": round(size, 1)})
        for mid in self._models:
            if mid not in seen:
                out.append({"model": mid, "loaded": True, "is_default": mid == default_model, "size_mb": 0})
        return out

    def _find_cache_path(self, model_id: str) -> Path | None:
        """``_find_cache_path`` (src/backends/faster_whisper.py:174-195): ``models--Org--Name``,
        and with ``STT_MODEL_DIR`` set also ``<dir>/<Name>``."""
        root = self._cache_root()
        if not root.exists():
            return None
        p = root / ("models--" + model_id.replace("/", "--"))
        if p.exists():
            return p
        if self._settings.get("stt_model_dir", None):
            p = root / model_id.split("/")[-1]
            if p.exists():
                return p
        return None

    def delete_cached_model(self, model_id: str) -> bool:
        p = self._find_cache_path(model_id)
        if p is not None:
            shutil.rmtree(p)
            return True
        return False

    def is_model_cached(self, model_id: str) -> bool:
        return self._find_cache_path(model_id) is not None

    # ------------------------------------------------------------ inference
    def _ensure_model(self, model_id: str) -> _Model:
        if model_id not in self._models:
            self.load_model(model_id)
        self._last_used[model_id] = time.time()
        return self._models[model_id]

    def _run_inference(self, audio: bytes, model_id: str, task: str = "transcribe", language: str | None = None,
                       response_format: str = "json", temperature: float = 0.0,
                       prompt: str | None = None) -> dict[str, Any]:
        m = self._ensure_model(model_id)
        pcm = decode_audio_bytes(audio)
        opts = TranscribeOptions(task=task, language=language if (language and task == "transcribe") else None,
                                 initial_prompt=prompt or None, temperature=float(temperature or 0.0),
                                 beam_size=int(os.environ.get("STT_HIP_BEAM_SIZE", "5")),
                                 best_of=int(os.environ.get("STT_HIP_BEST_OF", "5")),
                                 tokens_per_second=self._length_control)
        res = m.runner.transcribe(pcm, opts)
        return shape_response(task, res, response_format)

    def transcribe(self, audio: bytes, model: str, language: str | None = None, response_format: str = "json",
                   temperature: float = 0.0, prompt: str | None = None) -> dict[str, Any]:
        return self._run_inference(audio, model, task="transcribe", language=language,
                                   response_format=response_format, temperature=temperature, prompt=prompt)

    def translate(self, audio: bytes, model: str, response_format: str = "json", temperature: float = 0.0,
                  prompt: str | None = None) -> dict[str, Any]:
        return self._run_inference(audio, model, task="translate", response_format=response_format,
                                   temperature=temperature, prompt=prompt)


def _default_engine_factory(dims, gpu: int, max_batch: int):
    from .engine import WhisperEngine

    return WhisperEngine(dims, device=gpu, max_batch=max_batch)


def install(router, backend: HipWhisperBackend | None = None) -> HipWhisperBackend:
    """Register the HIP backend into an open-speech ``BackendRouter`` (src/router.py)."""
    b = backend or HipWhisperBackend()
    router._backends["faster-whisper"] = b
    router._default_backend = b
    return b
