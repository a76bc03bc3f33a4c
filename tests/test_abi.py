"""The C-ABI library loads and exports every symbol include/alaya_hip.h declares (no GPU calls)."""

import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "alaya_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(alaya_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(native):
    lib = ctypes.CDLL(os.path.join(ROOT, "alayalite_amd", "libalaya_hip.so"))
    syms = declared_symbols()
    assert len(syms) >= 15
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_library_has_gfx950_code_object(native):
    data = open(os.path.join(ROOT, "alayalite_amd", "libalaya_hip.so"), "rb").read()
    assert b"gfx950" in data


def test_no_device_fails_loudly(native):
    if native.device_count() > 0:
        return
    import pytest

    with pytest.raises(RuntimeError, match="no HIP device"):
        native.DeviceIndex(0)
