"""Model id -> weights + dims + tokenizer, offline only.

Mirrors where the reference finds models (``src/backends/faster_whisper.py:93-208``:
``STT_MODEL_DIR`` or the HuggingFace hub cache, ``models--Org--Name`` dirs) and
what ``WhisperModel(model_id, ...)`` accepts (an id or a local directory).
Supported on-disk formats:

* a transformers Whisper checkpoint: ``config.json`` + ``model.safetensors``
  (e.g. ``openai/whisper-large-v3-turbo``), optional ``tokenizer.json``;
* ``random:<preset>[:<seed>]`` — deterministic random weights at a preset's dims
  (``large-v3-turbo``, ``tiny-test``, ``micro-test``) for benchmarking and tests.

* a CTranslate2 directory: ``model.bin`` (+ ``tokenizer.json``) — the format of the
  reference's default ``deepdml/faster-whisper-large-v3-turbo-ct2`` (``ct2.py``).

Nothing here downloads.
"""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass

import numpy as np

from .dims import PRESETS, WhisperDims
from .weights import dims_from_hf_config, from_hf_state_dict


@dataclass
class ModelSource:
    model_id: str
    dims: WhisperDims
    kind: str               # "random" | "hf" | "ct2"
    path: str | None = None
    seed: int = 0
    tokenizer_json: str | None = None


def cache_dirs(model_dir: str | None) -> list[str]:
    out = []
    if model_dir:
        out.append(model_dir)
    for env in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE"):
        if os.environ.get(env):
            out.append(os.environ[env])
    out.append(os.path.join(os.path.expanduser("~"), ".cache", "huggingface", "hub"))
    return out


def _snapshot_dirs(model_id: str, model_dir: str | None) -> list[str]:
    cands = []
    if os.path.isdir(model_id):
        cands.append(model_id)
    safe = "models--" + model_id.replace("/", "--")
    for root in cache_dirs(model_dir):
        cands.extend(sorted(glob.glob(os.path.join(root, safe, "snapshots", "*"))))
        p = os.path.join(root, model_id.split("/")[-1])
        if os.path.isdir(p):
            cands.append(p)
    return cands


def resolve(model_id: str, model_dir: str | None = None) -> ModelSource:
    if model_id.startswith("random:"):
        parts = model_id.split(":")
        preset = parts[1] if len(parts) > 1 else "large-v3-turbo"
        if preset not in PRESETS:
            raise ValueError(f"unknown preset {preset!r}; choose from {sorted(PRESETS)}")
        seed = int(parts[2]) if len(parts) > 2 else 0
        return ModelSource(model_id, PRESETS[preset], "random", seed=seed)
    for d in _snapshot_dirs(model_id, model_dir):
        cfg = os.path.join(d, "config.json")
        st = sorted(glob.glob(os.path.join(d, "model*.safetensors")))
        tok = os.path.join(d, "tokenizer.json")
        if os.path.exists(cfg) and st:
            with open(cfg) as fh:
                dims = dims_from_hf_config(json.load(fh))
            return ModelSource(model_id, dims, "hf", path=d, tokenizer_json=tok if os.path.exists(tok) else None)
        mb = os.path.join(d, "model.bin")
        if os.path.exists(mb):
            from .ct2 import dims_from_ct2, read_model_bin

            v, _ = read_model_bin(mb)
            return ModelSource(model_id, dims_from_ct2(v), "ct2", path=d,
                               tokenizer_json=tok if os.path.exists(tok) else None)
    raise FileNotFoundError(f"model {model_id!r} not found locally (searched {cache_dirs(model_dir)}); "
                            "this backend never downloads")


def load_weights(src: ModelSource) -> dict | None:
    """Canonical weights for a resolved source (None for random init)."""
    if src.kind == "hf":
        return load_hf_weights(src)
    if src.kind == "ct2":
        from .ct2 import ct2_to_canonical, read_model_bin

        v, aliases = read_model_bin(os.path.join(src.path, "model.bin"))
        return ct2_to_canonical(v, aliases, src.dims)
    return None


def load_hf_weights(src: ModelSource) -> dict:
    from safetensors.numpy import load_file

    sd = {}
    for f in sorted(glob.glob(os.path.join(src.path, "model*.safetensors"))):
        for k, v in load_file(f).items():
            sd[k] = v.astype(np.float32) if v.dtype != np.float32 else v
    if "model.decoder.embed_tokens.weight" not in sd:
        raise ValueError("not a Whisper checkpoint (no model.decoder.embed_tokens.weight)")
    return from_hf_state_dict(sd, src.dims)
