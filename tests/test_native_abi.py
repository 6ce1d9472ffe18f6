"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed)."""

from __future__ import annotations

import ctypes
import re
import subprocess

import pytest

from tests.conftest import ROOT


def declared_symbols() -> set[str]:
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(taxi2_[a-z_]+)\s*\(", text))
    return names


def test_header_declares_entry_points():
    names = declared_symbols()
    assert {"taxi2_ctx_create", "taxi2_all_pairs", "taxi2_closest", "taxi2_align_strings"} <= names


def test_library_exports_every_declared_symbol():
    from taxi2_amd import _native

    lib = _native.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert set(_native.EXPORTS) == declared_symbols()
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native.LIB_PATH)], capture_output=True, text=True)
    exported = set(re.findall(r" T (taxi2_\w+)", out.stdout))
    assert declared_symbols() <= exported


def test_library_is_gfx950():
    from taxi2_amd import _native

    data = _native.LIB_PATH.read_bytes()
    assert b"gfx950" in data
    assert "gfx950" in _native.version()


def test_no_cpu_fallback_without_gpu():
    """Constructing an engine without a visible GPU fails loudly."""
    from taxi2_amd import _native

    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_native.NativeError):
        _native.Engine(0)


def test_error_path_through_abi():
    """Errors come back as status codes + taxi2_last_error, never an abort."""
    from taxi2_amd import _native

    lib = _native.load_library()
    assert lib.taxi2_set_destroy(None, 0) == -1
    assert b"null" in lib.taxi2_last_error(None)
    ctx = ctypes.c_void_p()
    if _native.device_count() == 0:
        assert lib.taxi2_ctx_create(0, ctypes.byref(ctx)) != 0
