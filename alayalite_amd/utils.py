"""Vector file IO, ground truth and recall (mirrors alayalite/utils.py, python/src/alayalite/utils.py:26-115)."""

from __future__ import annotations

import hashlib

import numpy as np

__all__ = ["load_fvecs", "load_ivecs", "calc_recall", "calc_gt", "calc_gt_device", "md5"]


def _load_vecs(file_path, dtype):
    raw = np.fromfile(file_path, dtype=np.int32)
    if raw.size == 0:
        return np.zeros((0, 0), dtype)
    dim = int(raw[0])
    rows = raw.reshape(-1, dim + 1)
    return rows[:, 1:].copy().view(dtype)


def load_fvecs(file_path):
    """fvecs: per vector an int32 dimension followed by that many float32 values."""
    return _load_vecs(file_path, np.float32)


def load_ivecs(file_path):
    """ivecs: per vector an int32 dimension followed by that many int32 values."""
    return _load_vecs(file_path, np.int32)


def calc_recall(result, gt_data):
    """Mean |result_i ∩ gt_i| / k over the rows (utils.py:78-84)."""
    rows, cols = result.shape
    hits = sum(len(set(result[i].tolist()) & set(gt_data[i].tolist())) for i in range(rows))
    return 1.0 * hits / (rows * cols)


def calc_gt(data, query, topk):
    """Exact top-k by float64 L2 (utils.py:99-105)."""
    gt = np.zeros((query.shape[0], topk), dtype=np.int32)
    base = data.astype(np.float64)
    for i in range(query.shape[0]):
        d = np.linalg.norm(base - query[i].astype(np.float64), axis=1)
        gt[i] = np.argsort(d)[:topk]
    return gt


def calc_gt_device(data, query, topk, device=0):
    """Exact top-k L2 on the MI355X: the flat MFMA path (IndexType::FLAT has no implementation in the
    reference; this is its exact search, find_exact_gt in include/utils/evaluate.hpp:29-62: the f32
    l2_sqr metric, ties by id).  Any dimension, 1 <= topk <= 224.  Returns (ids int32, distances
    float32).  Differs from calc_gt (float64 norms) only where two rows tie within f32 rounding."""
    from . import _native

    data = np.ascontiguousarray(data, dtype=np.float32)
    query = np.ascontiguousarray(query, dtype=np.float32)
    ix = _native._ext.DeviceIndex(device)
    ix.set_base(data, 0)
    ids, dists, _ = ix.flat_search(query, topk)
    return ids.astype(np.int32), dists


def md5(arr, chunk_size=1024 * 1024):
    h = hashlib.md5()
    data = arr.tobytes()
    for i in range(0, len(data), chunk_size):
        h.update(data[i:i + chunk_size])
    return h.hexdigest()
