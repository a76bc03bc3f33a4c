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


def test_import_starts_no_gpu_runtime():
    """Importing the package loads torch's libraries (so the engine's HIP soname resolves to the
    runtime torch uses) but calls nothing on the device: torch.cuda.is_available() is never called
    and torch stays uninitialised (a fork or exec after import must stay safe)."""
    import subprocess
    import sys

    code = (
        "import torch, torch.cuda\n"
        "calls = []\n"
        "real = torch.cuda.is_available\n"
        "torch.cuda.is_available = lambda *a, **k: calls.append(1) or real(*a, **k)\n"
        "import alayalite_amd\n"
        "assert calls == [], calls\n"
        "assert not torch.cuda.is_initialized()\n"
        "print('ok')\n")
    env = dict(os.environ)
    env.pop("ALAYA_SKIP_TORCH_INIT", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_build_provenance_matches_tree(native):
    """The library carries the hash of the sources it was compiled from (alaya_build_info), and the
    in-tree library is current: built from the sources in this tree."""
    lib = ctypes.CDLL(os.path.join(ROOT, "alayalite_amd", "libalaya_hip.so"))
    lib.alaya_build_info.restype = ctypes.c_char_p
    info = lib.alaya_build_info().decode()
    assert info.startswith("source=") and "arch=gfx950" in info, info
    from alayalite_amd import _native

    prov = _native.build_provenance()
    assert prov["library"] == info
    assert prov["library_matches_tree"], prov
