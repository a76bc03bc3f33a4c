"""Index: one vector index whose search runs on the MI355X (mirrors alayalite/index.py,
python/src/alayalite/index.py:35-231; same signatures, same ValueError/RuntimeError behaviour)."""

from __future__ import annotations

import os

import numpy as np

from ._native import PyIndexInterface as _PyIndexInterface
from .common import VectorLike, VectorLikeBatch, _assert
from .schema import IndexParams, load_schema


class Index:
    """A vector index: ``fit`` builds the HNSW graph (host) and uploads rows + graph to HBM; all
    ``search`` / ``batch_search`` calls run the device graph search kernel."""

    def __init__(self, name: str = "default", params: IndexParams = None):
        self.__name = name
        self.__params = params if params is not None else IndexParams()
        self.__index = None
        self.__is_initialized = False
        self.__dim = None

    def get_params(self) -> IndexParams:
        return self.__params

    def get_data_by_id(self, vector_id: int) -> VectorLike:
        return self.__index.get_data_by_id(vector_id)

    def fit(self, vectors: VectorLikeBatch, ef_construction: int = 100, num_threads: int = 1,
            builder: str = "host"):
        """index.py:75-99.  builder="host" builds the graph with the reference's HNSWBuilder restated
        on the host (num_threads=1 gives the reference's graph exactly); builder="gpu" builds it on the
        MI355X by batched insertion (alaya_index_build_graph) -- same algorithm, orders of magnitude
        faster at 1M+ rows, graph not identical to the sequential one."""
        _assert(builder in ("host", "gpu"), "builder must be 'host' or 'gpu'")
        if self.__is_initialized:
            raise RuntimeError("An index can be only fitted once")
        _assert(vectors.ndim == 2, "vectors must be a 2D array")
        data_type = np.array(vectors).dtype
        if self.__params.data_type is None:
            self.__params.data_type = data_type
        elif self.__params.data_type != data_type:
            raise ValueError(f"Data type mismatch: {self.__params.data_type} vs {data_type}")
        self.__params.fill_none_values()
        self.__dim = vectors.shape[1]
        self.__index = _PyIndexInterface(self.__params.to_cpp_params())
        self.__is_initialized = True
        self.__index.fit(vectors, ef_construction, num_threads, builder)

    def insert(self, vectors: VectorLike, ef: int = 100):
        _assert(self.__index is not None, "Index is not init yet")
        _assert(vectors.ndim == 1, "vectors must be a 1D array")
        _assert(vectors.shape[0] == self.__dim,
                "vectors dimension must match the dimension of the vectors used to fit the index."
                f"fit data dimension: {self.__dim}, vectors dimension: {vectors.shape[0]}")
        ret = self.__index.insert(vectors, ef)
        full = ret == -1 or (self.__params.id_type == np.uint32 and ret == 0xFFFFFFFF) or (
            self.__params.id_type == np.uint64 and ret == 0xFFFFFFFFFFFFFFFF)
        if full:
            raise RuntimeError("The index is full, cannot insert more vectors")
        return ret

    def remove(self, vector_id: int) -> None:
        _assert(self.__index is not None, "Index is not init yet")
        self.__index.remove(vector_id)

    def _check_queries(self, queries, ndim: int, what: str):
        _assert(self.__index is not None, "Index is not init yet")
        _assert(queries.ndim == ndim, f"{what} must be a {ndim}D array")
        got = queries.shape[-1]
        _assert(got == self.__dim,
                "query dimension must match the dimension of the vectors used to fit the index."
                f"fit data dimension: {self.__dim}, query dimension: {got}")

    def search(self, query: VectorLike, topk: int, ef_search: int = 100) -> VectorLike:
        self._check_queries(query, 1, "query")
        return self.__index.search(query, topk, ef_search)

    def batch_search(self, queries: VectorLikeBatch, topk: int, ef_search: int = 100,
                     num_threads: int = 1) -> VectorLikeBatch:
        self._check_queries(queries, 2, "queries")
        return self.__index.batch_search(queries, topk, ef_search, num_threads)

    def batch_search_with_distance(self, queries: VectorLikeBatch, topk: int, ef_search: int = 100,
                                   num_threads: int = 1):
        self._check_queries(queries, 2, "queries")
        return self.__index.batch_search_with_distance(queries, topk, ef_search, num_threads)

    def get_dim(self):
        return self.__dim

    def get_dtype(self):
        return self.__params.data_type

    # ---- engine extras (not in the reference API) -------------------------------------------
    def native(self):
        """The underlying PyIndexInterface (device counters, graph arrays, tuning)."""
        return self.__index

    def save(self, url) -> dict:
        os.makedirs(url, exist_ok=True)
        p = self.__params
        self.__index.save(p.index_path(url), p.data_path(url), p.quant_path(url))
        return {"type": "index", "index": p.to_json_dict()}

    @classmethod
    def load(cls, url, name):
        index_url = os.path.join(url, name)
        if not os.path.exists(index_url):
            raise RuntimeError("The index file does not exist")
        params = IndexParams.from_str_dict(load_schema(os.path.join(index_url, "schema.json"))["index"])
        instance = cls(name, params)
        instance.__index = _PyIndexInterface(params.to_cpp_params())
        instance.__index.load(params.index_path(index_url), params.data_path(index_url), params.quant_path(index_url))
        instance.__is_initialized = True
        instance.__dim = instance.__index.get_data_dim()
        return instance
