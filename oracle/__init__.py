"""TEST INFRASTRUCTURE ONLY: ctypes view of the CPU restatement (oracle/liboracle.so).

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package.  The product package ``alayalite_amd`` never imports it.  See oracle.h for the reference
file:line each function restates.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

L2, IP, COS = 0, 1, 2


class OrcIndex(C.Structure):
    _fields_ = [
        ("base", C.c_void_p),
        ("n", C.c_uint64),
        ("dim", C.c_uint32),
        ("stride", C.c_uint32),
        ("valid", C.c_void_p),
        ("metric", C.c_int),
        ("l0", C.c_void_p),
        ("R", C.c_uint32),
        ("levels", C.c_void_p),
        ("upper_off", C.c_void_p),
        ("upper_edges", C.c_void_p),
        ("upper_R", C.c_uint32),
        ("ep", C.c_uint32),
        ("space", C.c_int),
        ("codes", C.c_void_p),
        ("code_stride", C.c_uint32),
        ("sq_min", C.c_void_p),
        ("sq_max", C.c_void_p),
        ("sq8_variant", C.c_int),
        ("generic", C.c_int),
    ]


class OrcCounters(C.Structure):
    _fields_ = [
        ("n_dist", C.c_uint64),
        ("n_expand", C.c_uint64),
        ("n_dist_upper", C.c_uint64),
        ("n_hops_upper", C.c_uint64),
    ]


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc only, no GPU)."""
    srcs = [os.path.join(_HERE, f) for f in ("oracle.cpp", "oracle_build.cpp", "oracle.h", "Makefile")]
    if force or not os.path.exists(_LIB_PATH) or any(os.path.getmtime(_LIB_PATH) < os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(_LIB_PATH)
        f = C.c_float
        p = C.c_void_p
        sz = C.c_size_t
        for name in ("orc_l2_f32", "orc_ip_f32", "orc_l2_f32_avx2", "orc_ip_f32_avx2"):
            getattr(_lib, name).restype = f
            getattr(_lib, name).argtypes = [p, p, sz]
        for name in ("orc_l2_generic", "orc_ip_generic"):
            getattr(_lib, name).restype = f
            getattr(_lib, name).argtypes = [p, p, sz, C.c_int]
        _lib.orc_normalize.argtypes = [p, sz]
        _lib.orc_pool_new.restype = p
        _lib.orc_pool_new.argtypes = [C.c_uint32, C.c_int]
        _lib.orc_pool_free.argtypes = [p]
        _lib.orc_pool_insert.restype = C.c_int
        _lib.orc_pool_insert.argtypes = [p, C.c_uint32, f]
        _lib.orc_pool_pop.restype = C.c_uint32
        _lib.orc_pool_pop.argtypes = [p]
        _lib.orc_pool_top.restype = C.c_uint32
        _lib.orc_pool_top.argtypes = [p]
        _lib.orc_pool_has_next.restype = C.c_int
        _lib.orc_pool_has_next.argtypes = [p]
        _lib.orc_pool_size.restype = sz
        _lib.orc_pool_size.argtypes = [p]
        _lib.orc_pool_id.restype = C.c_uint32
        _lib.orc_pool_id.argtypes = [p, sz]
        _lib.orc_pool_dist.restype = f
        _lib.orc_pool_dist.argtypes = [p, sz]
        _lib.orc_search.argtypes = [C.POINTER(OrcIndex), p, C.c_uint32, C.c_uint32, p, p, C.POINTER(OrcCounters)]
        _lib.orc_batch_search_coro.restype = C.c_double
        _lib.orc_batch_search_coro.argtypes = [
            C.POINTER(OrcIndex), p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, p, p, p]
        _lib.orc_rerank.argtypes = [C.POINTER(OrcIndex), p, p, C.c_uint32, C.c_uint32, p, p]
        _lib.orc_updater_new.restype = p
        _lib.orc_updater_new.argtypes = [C.POINTER(OrcIndex), C.c_uint64]
        _lib.orc_updater_free.argtypes = [p]
        _lib.orc_updater_view.restype = C.POINTER(OrcIndex)
        _lib.orc_updater_view.argtypes = [p]
        _lib.orc_updater_insert.restype = C.c_int64
        _lib.orc_updater_insert.argtypes = [p, p, p, C.c_uint32]
        _lib.orc_updater_remove.argtypes = [p, C.c_uint32]
        _lib.orc_batch_rerank.restype = C.c_double
        _lib.orc_batch_rerank.argtypes = [C.POINTER(OrcIndex), p, C.c_uint64, p, C.c_uint32, C.c_uint32, p, p]
        _lib.orc_exact_gt.restype = C.c_double
        _lib.orc_exact_gt.argtypes = [p, C.c_uint64, C.c_uint32, p, C.c_uint64, C.c_uint32, C.c_uint32, p]
        _lib.orc_sq8_fit.argtypes = [p, C.c_uint64, C.c_uint32, p, p]
        _lib.orc_sq8_encode.argtypes = [p, C.c_uint32, p, p, p]
        for name in ("orc_sq8_l2", "orc_sq8_ip"):
            getattr(_lib, name).restype = f
            getattr(_lib, name).argtypes = [p, p, sz, p, p, C.c_int]
        _lib.orc_hnsw_build.restype = p
        _lib.orc_hnsw_build.argtypes = [p, C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                        C.c_uint64]
        _lib.orc_hnsw_upper_slots.restype = C.c_uint64
        _lib.orc_hnsw_upper_slots.argtypes = [p]
        _lib.orc_hnsw_export.argtypes = [p, p, p, p, p, p]
        _lib.orc_hnsw_free.argtypes = [p]
        _lib.orc_cpu_has_avx2_fma.restype = C.c_int
        _lib.orc_cpu_has_avx512f.restype = C.c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


# ---------------------------------------------------------------------------------------------
def l2(x, y) -> np.float32:
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    return np.float32(lib().orc_l2_f32(_ptr(x), _ptr(y), x.shape[0]))


def ip(x, y) -> np.float32:
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    return np.float32(lib().orc_ip_f32(_ptr(x), _ptr(y), x.shape[0]))


def dist(metric: int, x, y) -> np.float32:
    return l2(x, y) if metric == L2 else ip(x, y)


def normalize(v: np.ndarray) -> np.ndarray:
    v = np.array(v, np.float32, copy=True)
    lib().orc_normalize(_ptr(v), v.shape[0])
    return v


class Pool:
    """LinearPool<float, uint32> (query_utils.hpp:236-312)."""

    def __init__(self, n: int, capacity: int):
        self._h = lib().orc_pool_new(n, capacity)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_pool_free(self._h)
            self._h = None

    def insert(self, i, d):
        return bool(lib().orc_pool_insert(self._h, i, d))

    def pop(self):
        return lib().orc_pool_pop(self._h)

    def top(self):
        return lib().orc_pool_top(self._h)

    def has_next(self):
        return bool(lib().orc_pool_has_next(self._h))

    def size(self):
        return lib().orc_pool_size(self._h)

    def id(self, i):
        return lib().orc_pool_id(self._h, i)

    def dist(self, i):
        return lib().orc_pool_dist(self._h, i)


def exact_gt(base, queries, k, num_threads=1):
    """find_exact_gt (evaluate.hpp:29-62) restated; returns (ids[nq, k], seconds)."""
    b = np.ascontiguousarray(base, np.float32)
    q = np.ascontiguousarray(queries, np.float32)
    ids = np.zeros((q.shape[0], k), np.uint32)
    sec = lib().orc_exact_gt(_ptr(b), b.shape[0], b.shape[1], _ptr(q), q.shape[0], k, num_threads, _ptr(ids))
    return ids, sec


class IndexView:
    """Host arrays of one index (base rows + HNSW graph) in the layout orc_index expects."""

    def __init__(self, base, l0, levels, upper_off, upper_edges, upper_R, ep, metric=L2, valid=None,
                 sq8=None, generic=False):
        """sq8 = (codes[n, d] uint8, min[d], max[d], variant) switches the search space to SQ8Space.
        generic = True: the rows are a non-float DataType cast to float, compared with the generic
        l2_sqr<T>/ip_sqr<T> branch (distance_l2.ipp:735-741) instead of the AVX2 float kernel."""
        self.base = np.ascontiguousarray(base, np.float32)
        self.l0 = np.ascontiguousarray(l0, np.uint32)
        self.levels = None if levels is None else np.ascontiguousarray(levels, np.uint32)
        self.upper_off = None if upper_off is None else np.ascontiguousarray(upper_off, np.uint64)
        self.upper_edges = None if upper_edges is None else np.ascontiguousarray(upper_edges, np.uint32)
        if self.upper_edges is not None and self.upper_edges.size == 0:
            self.upper_edges = np.zeros(1, np.uint32)
        self.valid = None if valid is None else np.ascontiguousarray(valid, np.uint8)
        self.s = OrcIndex(
            base=_ptr(self.base), n=self.base.shape[0], dim=self.base.shape[1], stride=self.base.shape[1],
            valid=_ptr(self.valid), metric=metric, l0=_ptr(self.l0), R=self.l0.shape[1],
            levels=_ptr(self.levels), upper_off=_ptr(self.upper_off), upper_edges=_ptr(self.upper_edges),
            upper_R=upper_R, ep=ep, generic=1 if generic else 0)
        if sq8 is not None:
            codes, mn, mx, variant = sq8
            self.codes = np.ascontiguousarray(codes, np.uint8)
            self.sq_min = np.ascontiguousarray(mn, np.float32)
            self.sq_max = np.ascontiguousarray(mx, np.float32)
            self.s.space = 1
            self.s.codes = _ptr(self.codes)
            self.s.code_stride = self.codes.shape[1]
            self.s.sq_min = _ptr(self.sq_min)
            self.s.sq_max = _ptr(self.sq_max)
            self.s.sq8_variant = variant

    def rerank(self, query, search_ids, k, ef):
        """PyIndex::rerank on the raw f32 rows (index.hpp:450-488), Linux batch call shape."""
        q = np.ascontiguousarray(query, np.float32)
        src = np.ascontiguousarray(search_ids, np.uint32)
        ids = np.zeros(k, np.uint32)
        d = np.zeros(k, np.float32)
        lib().orc_rerank(C.byref(self.s), _ptr(q), _ptr(src), k, ef, _ptr(ids), _ptr(d))
        return ids, d

    def batch_rerank(self, queries, search_ids, k, ef):
        """The batch path's rerank loop (index.hpp:337-345); returns (ids, dists, seconds)."""
        q = np.ascontiguousarray(queries, np.float32)
        src = np.ascontiguousarray(search_ids, np.uint32)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        d = np.zeros((nq, k), np.float32)
        sec = lib().orc_batch_rerank(C.byref(self.s), _ptr(q), nq, _ptr(src), k, ef, _ptr(ids), _ptr(d))
        return ids, d, sec

    def search(self, query, k, ef, with_counters=False):
        q = np.ascontiguousarray(query, np.float32)
        ids = np.zeros(k, np.uint32)
        dists = np.zeros(k, np.float32)
        cnt = OrcCounters()
        lib().orc_search(C.byref(self.s), _ptr(q), k, ef, _ptr(ids), _ptr(dists), C.byref(cnt))
        if with_counters:
            return ids, dists, (cnt.n_dist, cnt.n_expand, cnt.n_dist_upper, cnt.n_hops_upper)
        return ids, dists

    def batch_search(self, queries, k, ef, num_threads=1):
        """Coroutine batch driver; returns (ids, dists, counters[nq,4] uint64, seconds)."""
        q = np.ascontiguousarray(queries, np.float32)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.uint32)
        dists = np.zeros((nq, k), np.float32)
        cnt = np.zeros((nq, 4), np.uint64)
        sec = lib().orc_batch_search_coro(C.byref(self.s), _ptr(q), nq, k, ef, num_threads,
                                          _ptr(ids), _ptr(dists), _ptr(cnt))
        return ids, dists, cnt, sec


class Updater:
    """GraphUpdateJob restated on a copy of an IndexView (graph_update_job.hpp:49-137)."""

    def __init__(self, view: IndexView, capacity: int):
        self._keep = view
        self._h = lib().orc_updater_new(C.byref(view.s), capacity)
        self.dim = view.base.shape[1]

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_updater_free(self._h)
            self._h = None

    def insert(self, search_query, row, ef):
        q = np.ascontiguousarray(search_query, np.float32)
        r = np.ascontiguousarray(row, np.float32)
        return int(lib().orc_updater_insert(self._h, _ptr(q), _ptr(r), ef))

    def remove(self, node):
        lib().orc_updater_remove(self._h, node)

    def _view(self):
        return lib().orc_updater_view(self._h).contents

    def n(self):
        return int(self._view().n)

    def l0(self):
        v = self._view()
        return np.ctypeslib.as_array(C.cast(v.l0, C.POINTER(C.c_uint32)), shape=(v.n, v.R)).copy()

    def search(self, query, k, ef):
        q = np.ascontiguousarray(query, np.float32)
        ids = np.zeros(k, np.uint32)
        d = np.zeros(k, np.float32)
        lib().orc_search(lib().orc_updater_view(self._h), _ptr(q), k, ef, _ptr(ids), _ptr(d), None)
        return ids, d


def build_hnsw(base, metric=L2, R=32, ef_construction=100, seed=100, generic=False):
    """HNSWBuilder::build_graph with one thread, restated (oracle_build.cpp).  Returns the graph as
    (l0[n, R], levels[n], upper_off[n], upper_edges, ep, upper_R) in the engine's Graph.arrays()
    layout."""
    b = np.ascontiguousarray(base, np.float32)
    n, dim = b.shape
    h = lib().orc_hnsw_build(_ptr(b), n, dim, metric, 1 if generic else 0, R, ef_construction, seed)
    try:
        slots = lib().orc_hnsw_upper_slots(h)
        l0 = np.zeros((n, R), np.uint32)
        levels = np.zeros(n, np.uint32)
        off = np.zeros(n, np.uint64)
        ue = np.zeros(max(slots, 1), np.uint32)
        ep = np.zeros(1, np.uint32)
        lib().orc_hnsw_export(h, _ptr(l0), _ptr(levels), _ptr(off), _ptr(ue), _ptr(ep))
    finally:
        lib().orc_hnsw_free(h)
    return l0, levels, off, ue[:slots], int(ep[0]), R


def sq8_fit(data):
    data = np.ascontiguousarray(data, np.float32)
    mn = np.zeros(data.shape[1], np.float32)
    mx = np.zeros(data.shape[1], np.float32)
    lib().orc_sq8_fit(_ptr(data), data.shape[0], data.shape[1], _ptr(mn), _ptr(mx))
    return mn, mx


def sq8_encode(rows, mn, mx):
    rows = np.ascontiguousarray(np.atleast_2d(rows), np.float32)
    out = np.zeros(rows.shape, np.uint8)
    for i in range(rows.shape[0]):
        lib().orc_sq8_encode(_ptr(rows[i]), rows.shape[1], _ptr(mn), _ptr(mx), _ptr(out[i]))
    return out


def sq8_dist(metric, x, y, mn, mx, variant):
    x = np.ascontiguousarray(x, np.uint8)
    y = np.ascontiguousarray(y, np.uint8)
    mn = np.ascontiguousarray(mn, np.float32)
    mx = np.ascontiguousarray(mx, np.float32)
    fn = lib().orc_sq8_l2 if metric == L2 else lib().orc_sq8_ip
    return np.float32(fn(_ptr(x), _ptr(y), x.shape[0], _ptr(mn), _ptr(mx), variant))


def sq8_host_variant() -> int:
    """get_l2_sqr_sq8_func / get_ip_sqr_sq8_func choice on this host (distance_l2.ipp:694-708)."""
    if lib().orc_cpu_has_avx512f():
        return 2
    if lib().orc_cpu_has_avx2_fma():
        return 1
    return 0
