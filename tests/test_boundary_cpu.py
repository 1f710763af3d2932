"""C-ABI library: loads here (no GPU needed) and exports every symbol include/osw.h declares."""
import ctypes
import os
import re

import pytest

from open_speech_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "osw.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(osw_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert header_functions() == sorted(_lib.EXPORTED)


def test_library_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libosw_hip.so not built")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name


def test_version_without_gpu():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libosw_hip.so not built")
    lib = _lib.load()
    assert b"gfx950" in lib.osw_version()


def test_struct_sizes_match_header():
    # sizes computed from the C declarations (x86-64 SysV)
    assert ctypes.sizeof(_lib.osw_dims) == 40
    assert ctypes.sizeof(_lib.osw_window) == 12
    assert ctypes.sizeof(_lib.osw_window_result) == 64
    assert ctypes.sizeof(_lib.osw_profile) == 8 * 18


def test_product_path_has_no_cpu_fallback(tmp_path):
    """With the library absent, loading fails loudly (no silent eager fallback)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import osw_path; osw_path.load();"
            "from open_speech_amd import _lib\n"
            "try:\n    _lib.load()\nexcept RuntimeError as e:\n    print('RAISED', e)\n") % ROOT
    env = dict(__import__("os").environ, OSW_LIB=str(tmp_path / "missing.so"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "RAISED" in out.stdout and "no CPU fallback" in out.stdout
