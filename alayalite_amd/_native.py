"""Loads the in-tree native engine (``_alayalitepy`` over ``libalaya_hip.so``).

There is deliberately no fallback: if the HIP extension is missing this import fails loudly, and a
PyIndexInterface refuses to construct without a HIP device (the search path only exists on the GPU).
"""

from __future__ import annotations

import importlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def _runtime_order():
    """PyTorch-ROCm bundles its own HIP + HSA runtime (torch/lib) beside /opt/rocm's, which this
    engine links.  torch's libraries are loaded first (a plain ``import torch``), so the engine's
    HIP soname resolves to the runtime torch uses.  Nothing is initialised here: importing the
    package starts no GPU runtime (a later fork or exec stays safe), and the first device call --
    the engine's or torch's, in either order -- initialises the one runtime
    (tools/runtime_order_probe.py, profiles/r04/runtime_order.log).  ALAYA_SKIP_TORCH_INIT=1 skips
    the torch import for processes that never use torch (e.g. the sanitizer driver)."""
    if os.environ.get("ALAYA_SKIP_TORCH_INIT") == "1":
        return
    try:
        import torch  # noqa: F401  (loads the libraries; no device call)
    except ImportError:  # the engine itself does not need torch
        return


def _load():
    _runtime_order()
    try:
        return importlib.import_module("alayalite_amd._alayalitepy")
    except ImportError as exc:  # pragma: no cover - exercised only on a broken install
        raise ImportError(
            "alayalite_amd native extension is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            f"(looked in {_HERE}): {exc}") from exc


_ext = _load()

PyIndexInterface = _ext.PyIndexInterface
IndexParams = _ext.IndexParams
IndexType = _ext.IndexType
MetricType = _ext.MetricType
QuantizationType = _ext.QuantizationType
device_count = _ext.device_count


def build_provenance() -> dict:
    """Which sources the loaded library was compiled from (alaya_build_info) against the sources in
    this tree now: a stale library -- sources edited after the build, or a library from another
    tree -- shows as library_matches_tree = False in every bench line and smoke run."""
    from alayalite_amd import _build

    info = _ext.build_info()
    fields = dict(kv.split("=", 1) for kv in info.split() if "=" in kv)
    lib_hash = fields.get("source", "unknown")
    tree_hash = _build.source_hash()
    return {"library": info, "library_source_hash": lib_hash, "tree_source_hash": tree_hash,
            "library_matches_tree": lib_hash == tree_hash,
            "library_path": os.path.join(_HERE, "libalaya_hip.so")}
