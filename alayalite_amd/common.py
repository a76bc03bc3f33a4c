"""Types and argument validation shared by the SDK (mirrors alayalite/common.py of the reference:
python/src/alayalite/common.py:36-187).  Every validation failure raises ValueError, as the
reference's ``_assert`` does (common.py:185-187)."""

from __future__ import annotations

from pathlib import Path
from typing import Literal, Type, Union

import numpy as np
from numpy import typing as npt

from ._native import IndexType as _IndexType
from ._native import MetricType as _MetricType
from ._native import QuantizationType as _QuantizationType

IDType = Union[Type[np.uint64], Type[np.uint32]]
VectorDType = Union[Type[np.float32], Type[np.int8], Type[np.uint8], Type[np.float64], Type[np.int32], Type[np.uint32]]
DistanceMetric = Literal["euclidean", "l2", "ip", "cosine", "cos"]
QuantizationType = Literal[None, "none", "sq8", "sq4", "rabitq"]
IndexType = Literal["hnsw", "nsg", "fusion"]
VectorLike = npt.NDArray
VectorLikeBatch = npt.NDArray

_ID_TYPES = (np.uint64, np.uint32)
_DATA_TYPES = (np.float32, np.int8, np.uint8, np.float64, np.int32, np.uint32)
_METRICS = ("euclidean", "l2", "ip", "cosine", "cos")
_INDEX_TYPES = ("hnsw", "nsg", "fusion")
_QUANT_TYPES = (None, "none", "sq8", "sq4", "rabitq")

__all__ = [
    "VectorDType", "IDType", "valid_id_type", "valid_dtype", "valid_metric_type", "valid_index_type",
    "valid_capacity_type", "valid_quantization_type", "valid_max_nbrs",
]


def _assert(statement_eval: bool, message: str) -> None:
    if not statement_eval:
        raise ValueError(message)


def valid_dtype(dtype) -> np.dtype:
    _assert(any(np.can_cast(dtype, t) for t in _DATA_TYPES),
            "Vector dtype must be one of type {(np.single, np.float32), (np.byte, np.int8), "
            "(np.ubyte, np.uint8), (np.double, np.float64), (np.int32, np.int32), (np.uint32, np.uint32)}")
    return np.dtype(dtype)


def valid_id_type(id_type) -> np.dtype:
    _assert(any(np.can_cast(id_type, t) for t in _ID_TYPES), "ID dtype must be of one of type {(np.uint64), (np.uint32)}")
    return np.dtype(id_type)


def valid_capacity_type(capacity):
    _assert(capacity > 0, "Capacity must be greater than 0")
    return capacity


def assert_valid_metric_type(metric: str) -> None:
    _assert(metric.lower() in _METRICS, f"Distance metric must be one of {list(_METRICS)}")


def valid_metric_type(metric: str) -> _MetricType:
    assert_valid_metric_type(metric)
    m = metric.lower()
    if m == "ip":
        return _MetricType.IP
    if m in ("l2", "euclidean"):
        return _MetricType.L2
    return _MetricType.COS


def assert_valid_quantization_type(quantization_type) -> None:
    _assert(quantization_type is None or quantization_type.lower() in _QUANT_TYPES,
            f"Quantization type must be one of {list(_QUANT_TYPES)}")


def valid_quantization_type(quantization_type) -> _QuantizationType:
    assert_valid_quantization_type(quantization_type)
    q = "none" if quantization_type is None else quantization_type.lower()
    return {"none": _QuantizationType.NONE, "sq8": _QuantizationType.SQ8,
            "sq4": _QuantizationType.SQ4, "rabitq": _QuantizationType.RABITQ}[q]


def assert_valid_index_type(index: str) -> None:
    _assert(index.lower() in _INDEX_TYPES, f"Index type must be one of {list(_INDEX_TYPES)}")


def valid_index_type(index: str) -> _IndexType:
    assert_valid_index_type(index)
    return {"hnsw": _IndexType.HNSW, "nsg": _IndexType.NSG, "fusion": _IndexType.FUSION}[index.lower()]


def valid_max_nbrs(max_nbrs):
    _assert(0 < max_nbrs < 1000, "Max neighbors must be greater than 0 and less than 1000")
    return max_nbrs


def valid_index_path(index_path: str) -> None:
    p = Path(index_path)
    _assert(p.exists() and p.is_dir(), "Index path must be a valid directory")


def valid_index_prefix(index_prefix: str) -> None:
    _assert(index_prefix != "", "Index prefix must not be empty")
