"""Import helper: the package directory is ``open-speech_amd/`` (a hyphenated name
that Python cannot import directly), so it is registered as ``open_speech_amd``."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "open-speech_amd")


def load():
    mod = sys.modules.get("open_speech_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "open_speech_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["open_speech_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
