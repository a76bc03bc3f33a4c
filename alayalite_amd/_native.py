"""Loads the in-tree native engine (``_alayalitepy`` over ``libalaya_hip.so``).

There is deliberately no fallback: if the HIP extension is missing this import fails loudly, and a
PyIndexInterface refuses to construct without a HIP device (the search path only exists on the GPU).
"""

from __future__ import annotations

import importlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
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
