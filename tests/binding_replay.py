"""INTEGRATION.md §2 -- the reference-side PyIndex binding -- replayed through the C ABI (ctypes).

Test infrastructure.  `LoadedIndex` holds what `PyIndex::load` (python/include/index.hpp:132-175)
leaves in a PyIndex for one index directory in the reference's on-disk layout, decoded with
tests/refformat.py:
  * graph_index_: Graph::load (graph.hpp:165-238);
  * build_space_: RawSpace::load (raw_space.hpp:219-250);
  * search_space_: SQ8Space::load (sq8_space.hpp:213-251), or the build space itself;
  * data_size_ = build_space_->data_size_, the row size in bytes (index.hpp:165), and data_dim_.
`ReplayPyIndex` transcribes the C++ of INTEGRATION.md §2 call for call: the same C-ABI functions,
the same arguments, in the same order.  The [Un] / [Qn] / [Sn] / [Dn] tags are the ones in the
comments there.  So the GPU test (tests/test_binding_replay.py) exercises the sequence a maintainer
would add to the reference, not the engine's own pybind module.  A CPU test keeps the two call
orders equal.  The reference's own helpers that the C++ calls (alaya::normalize,
data_utils.hpp:36-46) are stood in for by the oracle's restatement (oracle.normalize).
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

import refformat as rf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALAYA_DIST_GENERIC = 0x100
COS = 2


def load_lib():
    lib = C.CDLL(os.path.join(ROOT, "alayalite_amd", "libalaya_hip.so"))
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    sig = {
        "alaya_last_error": (C.c_char_p, []),
        "alaya_index_create": (i32, [i32, C.POINTER(vp)]),
        "alaya_index_destroy": (None, [vp]),
        "alaya_index_set_base": (i32, [vp, vp, u64, u32, i32, vp]),
        "alaya_graph_import": (i32, [u64, u32, vp, vp, vp, vp, u64, u32, u32, vp, u32, C.POINTER(vp)]),
        "alaya_index_set_graph": (i32, [vp, vp]),
        "alaya_graph_free": (None, [vp]),
        "alaya_index_set_sq8": (i32, [vp, vp, u64, u32, vp, vp, i32]),
        "alaya_index_batch_search": (i32, [vp, vp, u64, u32, u32, vp, vp, vp]),
        "alaya_index_batch_search_sq8": (i32, [vp, vp, vp, u64, u32, u32, i32, vp, vp, vp]),
        "alaya_index_info": (i32, [vp, C.POINTER(u64), C.POINTER(u32), C.POINTER(u32), C.POINTER(i32),
                                   C.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class LoadedIndex:
    """The state PyIndex::load leaves (index.hpp:132-175), for RawSpace<DataType> or SQ8Space<float>."""

    def __init__(self, index_file, data_file, quant_file, data_type, id_type):
        ib = np.dtype(id_type).itemsize
        self.data_type = np.dtype(data_type)
        self.id_type = np.dtype(id_type)
        g = rf.read_graph(index_file, ib)
        raw = rf.read_raw(data_file, ib, data_type)
        # build_space_ (RawSpace: metric_, data_size_ in bytes, dim_, item_cnt_, data_storage_)
        self.metric = raw["metric"]
        self.build_data_size = raw["data_size"]
        self.dim = raw["dim"]
        self.build_item_cnt = raw["item_cnt"]
        self.build_rows = raw["rows"]  # capacity x dim DataType: SequentialStorage slots (zero past pos)
        bits = np.zeros(((raw["capacity"] + 7) // 8) * 8, np.uint8)
        bits[: raw["capacity"]] = raw["valid"]
        self.bitmap = np.packbits(bits, bitorder="little")  # SequentialStorage::bitmap_
        # search_space_
        self.sq8 = quant_file is not None
        if self.sq8:
            s = rf.read_sq8(quant_file, ib, np.float32)
            self.search_item_cnt = s["item_cnt"]
            self.codes = s["rows"]
            self.sq_min, self.sq_max = s["min"], s["max"]
        else:
            self.search_item_cnt = self.build_item_cnt
        # graph_index_
        self.max_nbrs = g["max_nbrs"]
        self.graph_rows = g["rows"]  # capacity x max_nbrs IDType, -1 padded
        self.overlay = g["overlay"]
        self.eps = g["eps"]
        # PyIndex members set by load (index.hpp:165-166)
        self.data_size_ = self.build_data_size
        self.data_dim_ = self.dim


class ReplayPyIndex:
    """INTEGRATION.md §2's hip_upload / hip_queries / batch_search / batch_search_with_distance."""

    def __init__(self, lib, st: LoadedIndex, normalize, sq8_order):
        self.lib = lib
        self.st = st
        self.normalize = normalize  # alaya::normalize (data_utils.hpp:36-46) -- the oracle's restatement
        self.sq8_order = sq8_order  # alaya::simd::get_cpu_features().avx512f_ ? 2 : 1
        self.hip_ = None
        self.kHipSQ8 = st.sq8

    def hip_ok(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.alaya_last_error().decode())

    def hip_upload(self):
        st = self.st
        if self.kHipSQ8 and st.data_type != np.float32:
            raise RuntimeError("SQ8 over non-float rows has no device path")
        if self.hip_ is None:
            h = C.c_void_p()
            self.hip_ok(self.lib.alaya_index_create(0, C.byref(h)))  # [U0]
            self.hip_ = h
        n = st.search_item_cnt  # [U1] search_space_->get_data_num(), never data_size_
        dim = st.data_dim_
        rows = np.ascontiguousarray(st.build_rows[:n].astype(np.float32))  # [U2]
        metric = st.metric | (ALAYA_DIST_GENERIC if st.data_type != np.float32 else 0)
        self.hip_ok(self.lib.alaya_index_set_base(self.hip_, _p(rows), n, dim, metric, _p(st.bitmap)))  # [U3]
        R = st.max_nbrs
        l0 = np.ascontiguousarray(st.graph_rows[:n].astype(np.uint32))  # [U4] (64-bit -1 -> 0xffffffff)
        g = C.c_void_p()
        if st.overlay is not None:  # [U5]
            ov = st.overlay
            levels = np.zeros(n, np.uint32)
            off = np.zeros(n, np.uint64)
            upper = []
            for i in range(n):
                lst = ov["lists"][i]
                levels[i] = len(lst) // ov["max_nbrs"]
                off[i] = len(upper)
                upper.extend(int(x) & 0xFFFFFFFF for x in lst)
            upper = np.asarray(upper if upper else [0], np.uint32)
            self.hip_ok(self.lib.alaya_graph_import(n, R, _p(l0), _p(levels), _p(off), _p(upper), len(upper),
                                                    ov["max_nbrs"], ov["ep"], None, 0, C.byref(g)))
        else:  # [U5']
            eps = np.ascontiguousarray(st.eps.astype(np.uint32))
            self.hip_ok(self.lib.alaya_graph_import(n, R, _p(l0), None, None, None, 0, 0, 0, _p(eps), len(eps),
                                                    C.byref(g)))
        rc = self.lib.alaya_index_set_graph(self.hip_, g)  # [U6]
        self.lib.alaya_graph_free(g)
        self.hip_ok(rc)
        if self.kHipSQ8:  # [U7]
            codes = np.ascontiguousarray(st.codes[:n])
            mn = np.ascontiguousarray(st.sq_min, np.float32)
            mx = np.ascontiguousarray(st.sq_max, np.float32)
            self.hip_ok(self.lib.alaya_index_set_sq8(self.hip_, _p(codes), n, dim, _p(mn), _p(mx), self.sq8_order))

    def hip_queries(self, queries):
        """queries: the caller's array (normalised in place for COS, as the reference does)."""
        nq, dim = queries.shape
        q_sq8 = None
        if self.kHipSQ8 and self.st.metric == COS:
            q_sq8 = np.ascontiguousarray(queries, np.float32).copy()  # [Q1]
        if self.st.metric == COS:
            for i in range(nq):  # [Q2]
                queries[i] = self.normalize(queries[i])
        q = np.ascontiguousarray(queries.astype(np.float32))  # [Q3]
        return q, q_sq8

    def batch_search(self, queries, topk, ef):
        q, q_sq8 = self.hip_queries(queries)
        nq = q.shape[0]
        ids = np.zeros((nq, topk), np.uint32)
        if self.kHipSQ8:  # [S1]
            self.hip_ok(self.lib.alaya_index_batch_search_sq8(self.hip_, _p(q if q_sq8 is None else q_sq8), _p(q), nq,
                                                              topk, ef, 1, _p(ids), None, None))
        else:  # [S1']
            self.hip_ok(self.lib.alaya_index_batch_search(self.hip_, _p(q), nq, topk, ef, _p(ids), None, None))
        return ids.astype(self.st.id_type)

    def batch_search_with_distance(self, queries, topk, ef):
        q, q_sq8 = self.hip_queries(queries)
        nq = q.shape[0]
        ids = np.zeros((nq, topk), np.uint32)
        dists = np.zeros((nq, topk), np.float32)
        if self.kHipSQ8:  # [D1]
            self.hip_ok(self.lib.alaya_index_batch_search_sq8(self.hip_, _p(q if q_sq8 is None else q_sq8), _p(q), nq,
                                                              topk, ef, 0, _p(ids), None, None))
            return ids.astype(self.st.id_type), np.zeros((0, topk), np.float32)
        self.hip_ok(self.lib.alaya_index_batch_search(self.hip_, _p(q), nq, topk, ef, _p(ids), _p(dists), None))  # [D1']
        return ids.astype(self.st.id_type), dists

    def device_rows(self):
        """alaya_index_info's row count (introspection: what [U1] uploaded)."""
        n, d, s, m, b = C.c_uint64(), C.c_uint32(), C.c_uint32(), C.c_int(), C.c_uint64()
        self.hip_ok(self.lib.alaya_index_info(self.hip_, C.byref(n), C.byref(d), C.byref(s), C.byref(m), C.byref(b)))
        return int(n.value)

    def close(self):
        if self.hip_ is not None:
            self.lib.alaya_index_destroy(self.hip_)
            self.hip_ = None
