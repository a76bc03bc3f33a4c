"""Test-side codec of the reference's on-disk index formats, in numpy.

Written from the reference's writers and readers, independently of the engine's C++ (csrc/
hnsw_build.cpp save_graph/load_graph, pybind_module.cpp save_raw/load_raw/save_sq8/load_sq8), so
the tests can decode what the engine writes and hand-assemble files in the reference's layout:

  graph file        Graph::save/load (include/index/graph/graph.hpp:165-238): int32 nep, nep x IDType
                    eps, IDType max_nodes_, then max_nbrs_ -- a uint32 written with sizeof(IDType)
                    bytes (:179-180; for 64-bit ids the upper 4 bytes are the struct's padding),
                    SequentialStorage, then the OverlayGraph if any bytes remain (:233-236).
  SequentialStorage save/load (include/storage/sequential_storage.hpp:110-142): 5 x size_t
                    (item_size, aligned_item_size, capacity, pos, alignment), aligned_item_size x
                    capacity data bytes, ceil(capacity / 8) bitmap bytes (bit i % 8 of byte i / 8).
  OverlayGraph      save/load (overlay_graph.hpp:151-194): node_num_, max_nbrs_, ep_ with 4 bytes
                    each, then per node int32 cur = levels * max_nbrs and cur * 4 bytes of its IDType
                    list (for 64-bit ids: the first cur / 2 entries; load leaves the rest -1).
  raw data file     RawSpace::save/load (include/space/raw_space.hpp:219-250): int32 metric, uint32
                    data_size, uint32 dim, IDType item_cnt, delete_cnt, capacity, SequentialStorage of
                    DataType rows (rows stored after COS normalisation).
  SQ8 file          SQ8Space::save/load (include/space/sq8_space.hpp:213-251): the same header,
                    SequentialStorage of uint8 codes, then SQ8Quantizer::save (space/quant/sq8.hpp:
                    161-177): uint32 dim, dim x DataType min, dim x DataType max.
  schema.json       python/src/alayalite/schema.py:103-112, client.py:251-271.
"""

from __future__ import annotations

import json
import os

import numpy as np

U8 = np.uint8


class Reader:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        self.o = 0

    def take(self, n):
        if self.o + n > len(self.b):
            raise ValueError("truncated file")
        out = self.b[self.o:self.o + n]
        self.o += n
        return out

    def arr(self, dtype, count):
        dt = np.dtype(dtype)
        return np.frombuffer(self.take(dt.itemsize * count), dt).copy()

    def scalar(self, dtype):
        return self.arr(dtype, 1)[0]

    def eof(self):
        return self.o == len(self.b)


def _id_dtype(id_bytes):
    return np.uint32 if id_bytes == 4 else np.uint64


def read_storage(r: Reader, item_dtype):
    item, aligned, cap, pos, align = (int(x) for x in r.arr(np.uint64, 5))
    data = np.frombuffer(r.take(aligned * cap), U8).reshape(cap, aligned) if cap else np.zeros((0, aligned), U8)
    bitmap = np.frombuffer(r.take((cap + 7) // 8), U8)
    bits = np.unpackbits(bitmap, bitorder="little")[:cap].astype(bool)
    it = np.dtype(item_dtype)
    rows = np.ascontiguousarray(data[:, :item]).view(it) if cap else np.zeros((0, item // it.itemsize), it)
    return {"item_size": item, "aligned_item_size": aligned, "capacity": cap, "pos": pos, "alignment": align,
            "rows": rows, "valid": bits, "padding": data[:, item:]}


def write_storage(f, rows, capacity, pos, valid, fill, item_bytes):
    """SequentialStorage::save of `capacity` slots, `rows` (pos x item) in the first ones, the rest
    filled with `fill` (init(item_size, capacity, fill): Graph uses -1, spaces use 0)."""
    aligned = (item_bytes + 63) // 64 * 64
    np.array([item_bytes, aligned, capacity, pos, 64], np.uint64).tofile(f)
    data = np.full((capacity, aligned), fill, U8)
    raw = np.ascontiguousarray(rows).view(U8).reshape(len(rows), -1) if len(rows) else np.zeros((0, item_bytes), U8)
    data[: len(rows), :item_bytes] = raw
    data.tofile(f)
    bits = np.zeros(((capacity + 7) // 8) * 8, U8)
    bits[: len(valid)] = np.asarray(valid, bool)
    np.packbits(bits, bitorder="little").tofile(f)


# ---- graph -------------------------------------------------------------------------------------
def read_graph(path, id_bytes):
    idt = _id_dtype(id_bytes)
    r = Reader(path)
    nep = int(r.scalar(np.int32))
    eps = r.arr(idt, nep)
    max_nodes = int(r.scalar(idt))
    max_nbrs = int(r.arr(np.uint32, id_bytes // 4)[0])  # a uint32 written with sizeof(IDType) bytes
    st = read_storage(r, idt)
    out = {"eps": eps, "max_nodes": max_nodes, "max_nbrs": max_nbrs, **st, "overlay": None}
    if not r.eof():
        node_num = int(r.scalar(np.uint32))
        onbrs = int(r.scalar(np.uint32))
        ep = int(r.scalar(np.uint32))
        lists = []
        for _ in range(node_num):
            cur = int(r.scalar(np.int32))
            raw = r.take(cur * 4)
            lst = np.full(cur, np.iinfo(idt).max, idt)  # resize(cur, -1), then read cur * 4 bytes
            got = np.frombuffer(raw, idt) if id_bytes == 4 else np.frombuffer(raw[: (cur * 4) // 8 * 8], idt)
            lst[: len(got)] = got
            lists.append(lst)
        out["overlay"] = {"node_num": node_num, "max_nbrs": onbrs, "ep": ep, "lists": lists}
        assert r.eof(), "bytes after the overlay"
    return out


def write_graph(path, id_bytes, rows, capacity, valid=None, eps=(), overlay=None, max_nbrs_pad=0):
    """rows: n x R ids (-1 padded).  overlay: (ep, lists) with lists[i] the levels * R entries of node
    i (-1 padded) for i < capacity (missing / empty = level 0).  max_nbrs_pad: the value of the upper
    4 bytes of the 64-bit max_nbrs_ field (struct padding in the reference)."""
    idt = _id_dtype(id_bytes)
    rows = np.asarray(rows).astype(idt)
    n, R = rows.shape
    valid = np.ones(n, bool) if valid is None else np.asarray(valid, bool)
    with open(path, "wb") as f:
        np.array([len(eps)], np.int32).tofile(f)
        np.asarray(eps, idt).tofile(f)
        np.array([capacity], idt).tofile(f)
        if id_bytes == 4:
            np.array([R], np.uint32).tofile(f)
        else:
            np.array([R, max_nbrs_pad], np.uint32).tofile(f)
        write_storage(f, rows, capacity, n, valid, 0xFF, R * id_bytes)
        if overlay is not None:
            ep, lists = overlay
            np.array([capacity, R, ep], np.uint32).tofile(f)
            for i in range(capacity):
                lst = np.asarray(lists[i] if i < len(lists) else [], idt)
                np.array([len(lst)], np.int32).tofile(f)
                f.write(lst.tobytes()[: len(lst) * 4])


def overlay_lists(levels, upper_off, upper_edges, R):
    """The engine's overlay arrays -> per-node lists of levels * R ids."""
    out = []
    for i in range(len(levels)):
        lv = int(levels[i])
        out.append(np.asarray(upper_edges[int(upper_off[i]): int(upper_off[i]) + lv * R], np.uint32))
    return out


# ---- raw / SQ8 spaces --------------------------------------------------------------------------
def _read_space_header(r, id_bytes):
    idt = _id_dtype(id_bytes)
    metric = int(r.scalar(np.int32))
    data_size = int(r.scalar(np.uint32))
    dim = int(r.scalar(np.uint32))
    item_cnt, delete_cnt, capacity = (int(x) for x in r.arr(idt, 3))
    return {"metric": metric, "data_size": data_size, "dim": dim, "item_cnt": item_cnt, "delete_cnt": delete_cnt,
            "capacity": capacity}


def _write_space_header(f, id_bytes, metric, data_size, dim, item_cnt, delete_cnt, capacity):
    np.array([metric], np.int32).tofile(f)
    np.array([data_size, dim], np.uint32).tofile(f)
    np.array([item_cnt, delete_cnt, capacity], _id_dtype(id_bytes)).tofile(f)


def read_raw(path, id_bytes, dtype):
    r = Reader(path)
    hdr = _read_space_header(r, id_bytes)
    st = read_storage(r, dtype)
    assert r.eof(), "bytes after the raw storage"
    return {**hdr, **st}


def write_raw(path, id_bytes, metric, rows, capacity, valid=None, delete_cnt=0):
    rows = np.asarray(rows)
    n, dim = rows.shape
    valid = np.ones(n, bool) if valid is None else np.asarray(valid, bool)
    with open(path, "wb") as f:
        _write_space_header(f, id_bytes, metric, dim * rows.itemsize, dim, n, delete_cnt, capacity)
        write_storage(f, rows, capacity, n, valid, 0, dim * rows.itemsize)


def read_sq8(path, id_bytes, dtype):
    r = Reader(path)
    hdr = _read_space_header(r, id_bytes)
    st = read_storage(r, np.uint8)
    qdim = int(r.scalar(np.uint32))
    mn = r.arr(dtype, qdim)
    mx = r.arr(dtype, qdim)
    assert r.eof(), "bytes after the quantizer"
    return {**hdr, **st, "q_dim": qdim, "min": mn, "max": mx}


def write_sq8(path, id_bytes, metric, codes, capacity, mn, mx, dtype=np.float32):
    codes = np.asarray(codes, np.uint8)
    n, dim = codes.shape
    with open(path, "wb") as f:
        _write_space_header(f, id_bytes, metric, dim, dim, n, 0, capacity)
        write_storage(f, codes, capacity, n, np.ones(n, bool), 0, dim)
        np.array([dim], np.uint32).tofile(f)
        np.asarray(mn, dtype).tofile(f)
        np.asarray(mx, dtype).tofile(f)


def write_schema(index_dir, index_type, data_type, id_type, quantization_type, metric, capacity, max_nbrs):
    os.makedirs(index_dir, exist_ok=True)
    schema = {"type": "index", "index": {"index_type": index_type, "data_type": np.dtype(data_type).name,
                                         "id_type": np.dtype(id_type).name, "quantization_type": quantization_type,
                                         "metric": metric, "capacity": capacity, "max_nbrs": max_nbrs}}
    with open(os.path.join(index_dir, "schema.json"), "w", encoding="utf-8") as f:
        json.dump(schema, f, indent=4)
