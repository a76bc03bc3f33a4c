"""Index parameters and schema files (mirrors alayalite/schema.py, python/src/alayalite/schema.py:46-211)."""

from __future__ import annotations

import json
import os
import shutil
from dataclasses import dataclass

import numpy as np

from ._native import IndexParams as _IndexParams
from .common import (
    assert_valid_index_type,
    assert_valid_metric_type,
    assert_valid_quantization_type,
    valid_capacity_type,
    valid_dtype,
    valid_id_type,
    valid_index_type,
    valid_max_nbrs,
    valid_metric_type,
    valid_quantization_type,
)

__all__ = ["IndexParams", "load_schema", "save_schema"]

_DEFAULTS = {
    "index_type": "hnsw",
    "data_type": np.float32,
    "id_type": np.uint32,
    "quantization_type": "none",
    "metric": "l2",
    "capacity": 100000,  # schema.py:81-82 -- 1M/10M builds must pass capacity explicitly
    "max_nbrs": 32,
}


@dataclass
class IndexParams:
    """Parameters of one vector index (schema.py:46-56)."""

    index_type: str = None
    data_type: object = None
    id_type: object = None
    quantization_type: str = None
    metric: str = None
    capacity: int = None
    max_nbrs: int = None

    # on-disk layout: <folder>/{<index_type>_<metric>_<max_nbrs>.index, raw.data, <quant>.data}
    def index_path(self, folder_uri):
        return os.path.join(folder_uri, f"{self.index_type}_{self.metric}_{self.max_nbrs}.index")

    def data_path(self, folder_uri):
        return os.path.join(folder_uri, "raw.data")

    def quant_path(self, folder_uri):
        return "" if self.quantization_type == "none" else os.path.join(folder_uri, f"{self.quantization_type}.data")

    def fill_none_values(self):
        for key, value in _DEFAULTS.items():
            if getattr(self, key) is None:
                setattr(self, key, value)

    def to_cpp_params(self):
        # Like the reference (schema.py:86-101), max_nbrs is not forwarded: the graph degree is 32.
        return _IndexParams(
            index_type_=valid_index_type(self.index_type),
            data_type_=valid_dtype(self.data_type),
            id_type_=valid_id_type(self.id_type),
            quantization_type_=valid_quantization_type(self.quantization_type),
            metric_=valid_metric_type(self.metric),
            capacity_=valid_capacity_type(self.capacity),
        )

    def to_json_dict(self) -> dict:
        return {
            "index_type": self.index_type,
            "data_type": np.dtype(self.data_type).name,
            "id_type": np.dtype(self.id_type).name,
            "quantization_type": self.quantization_type,
            "metric": self.metric,
            "capacity": self.capacity,
            "max_nbrs": self.max_nbrs,
        }

    @classmethod
    def from_str_dict(cls, data: dict) -> "IndexParams":
        return cls(
            index_type=data["index_type"],
            data_type=np.dtype(data["data_type"]).type,
            id_type=np.dtype(data["id_type"]).type,
            quantization_type=data["quantization_type"],
            metric=data["metric"],
            capacity=data["capacity"],
            max_nbrs=data["max_nbrs"],
        )

    @classmethod
    def from_kwargs(cls, **kwargs) -> "IndexParams":
        out = cls()
        if kwargs.get("index_type") is not None:
            assert_valid_index_type(kwargs["index_type"])
            out.index_type = kwargs["index_type"]
        if kwargs.get("data_type") is not None:
            out.data_type = valid_dtype(kwargs["data_type"])
        if kwargs.get("id_type") is not None:
            out.id_type = valid_id_type(kwargs["id_type"])
        if kwargs.get("quantization_type") is not None:
            assert_valid_quantization_type(kwargs["quantization_type"])
            out.quantization_type = kwargs["quantization_type"]
        if kwargs.get("metric") is not None:
            assert_valid_metric_type(kwargs["metric"])
            out.metric = kwargs["metric"]
        if kwargs.get("capacity") is not None:
            out.capacity = valid_capacity_type(kwargs["capacity"])
        if kwargs.get("max_nbrs") is not None:
            out.max_nbrs = valid_max_nbrs(kwargs["max_nbrs"])
        return out


def load_schema(url) -> dict:
    if not os.path.exists(url):
        raise FileNotFoundError("The schema file does not exist!")
    with open(url, encoding="utf-8") as f:
        return json.load(f)


def save_schema(schema_url, schema_map):
    backup = schema_url + ".bak"
    shutil.copy2(schema_url, backup)
    with open(schema_url, "w", encoding="utf-8") as f:
        json.dump(schema_map, f, indent=4)
    os.remove(backup)


def _schema_type(url):
    path = os.path.join(url, "schema.json")
    return load_schema(path).get("type") if os.path.exists(path) else None


def is_index_url(url):
    return _schema_type(url) == "index"


def is_collection_url(url):
    return _schema_type(url) == "collection"
