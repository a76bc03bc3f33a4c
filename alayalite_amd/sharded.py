"""Base-range sharding across GPUs: one process per GPU, each rank holds rows
[lo, hi) of the base with its own HNSW graph, searches every query on its shard, and the per-shard
top-k (global ids + distances) are exchanged with one all_gather (RCCL over xGMI for "nccl", gloo
on CPU) and merged by (distance asc, global id asc) -- the pair<dist, id> order of
PyIndex::rerank (python/include/index.hpp:456-466); the reference itself has no multi-GPU path.
"""

from __future__ import annotations

import numpy as np


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


def merge_topk(all_ids, all_dists, k: int):
    """all_ids / all_dists: [nq, G*k] (torch).  Deterministic top-k by (dist, id)."""
    import torch

    o1 = torch.sort(all_ids, dim=1, stable=True).indices
    ids = torch.gather(all_ids, 1, o1)
    d = torch.gather(all_dists, 1, o1)
    o2 = torch.sort(d, dim=1, stable=True).indices[:, :k]
    return torch.gather(ids, 1, o2), torch.gather(d, 1, o2)


def pack_candidates(gid, dists):
    """(global id, f32 distance) -> one int64 whose signed order is (distance asc, id asc):
    the distance bits mapped to an order-preserving int32 (negatives' magnitude bits flipped,
    -0.0 folded into +0.0) in the high word, the id (< 2^32) in the low word."""
    import torch

    bits = (dists.to(torch.float32) + 0.0).contiguous().view(torch.int32).to(torch.int64)
    skey = torch.where(bits < 0, bits ^ 0x7FFFFFFF, bits)
    return (skey << 32) | (gid.to(torch.int64) & 0xFFFFFFFF)


def unpack_candidates(packed):
    import torch

    gid = packed & 0xFFFFFFFF
    skey = packed >> 32
    bits = torch.where(skey < 0, skey ^ 0x7FFFFFFF, skey).to(torch.int32)
    return gid, bits.view(torch.float32)


EMPTY = 0xFFFFFFFF  # an empty result slot of a shard search (shard_search_device): (EMPTY, FLT_MAX)


def to_global(local_ids, offset: int):
    """Shard-local ids -> global ids; empty slots (0xffffffff) stay empty."""
    import torch

    ids = local_ids.to(torch.int64) & 0xFFFFFFFF
    return torch.where(ids == EMPTY, ids, ids + offset)


def exchange_and_merge(local_ids, local_dists, offset: int, k: int, group=None):
    """local_ids: [nq, k] shard-local ids (int32/int64 tensor); returns merged global (ids, dists).
    One all_gather of packed (distance, id) keys and one sort: the smallest k keys are the top-k
    by (distance, global id).  Empty slots (id 0xffffffff, distance FLT_MAX) sort after every real
    candidate and appear in the result only when all shards together hold fewer than k."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    device = local_ids.device
    packed = pack_candidates(to_global(local_ids, offset), local_dists)
    if dist.get_backend(group) == "gloo" and device.type != "cpu":  # gloo gathers host tensors
        packed = packed.cpu()
    parts = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(parts, packed, group=group)
    best = torch.sort(torch.cat(parts, 1), dim=1).values[:, :k]
    ids, d = unpack_candidates(best)
    return ids.to(device), d.to(device)


def merge_reference(ids_per_shard, dists_per_shard, offsets, k):
    """numpy restatement of the merge (test checker)."""
    nq = ids_per_shard[0].shape[0]
    out_i = np.zeros((nq, k), np.int64)
    out_d = np.zeros((nq, k), np.float32)
    def glob(a, off):
        a = a.astype(np.int64) & 0xFFFFFFFF
        return np.where(a == EMPTY, a, a + off)

    for q in range(nq):
        ids = np.concatenate([glob(ids_per_shard[s][q], offsets[s]) for s in range(len(offsets))])
        ds = np.concatenate([dists_per_shard[s][q] for s in range(len(offsets))])
        o = np.lexsort((ids, ds))[:k]
        out_i[q], out_d[q] = ids[o], ds[o]
    return out_i, out_d


class ShardedIndex:
    """This rank's shard on its GPU: rows [lo, hi) of `base`, graph built on the shard."""

    def __init__(self, base, world: int, rank: int, device: int = 0, metric: int = 0, R: int = 32,
                 ef_construction: int = 100, num_threads: int = 1, graph=None):
        from ._native import _ext

        self.lo, self.hi = shard_range(base.shape[0], world, rank)
        self.rows = np.ascontiguousarray(base[self.lo:self.hi])
        self.graph = graph if graph is not None else _ext.Graph.build(self.rows, metric, R, ef_construction, num_threads, 100)
        self.index = _ext.DeviceIndex(device)
        self.index.set_base(self.rows, metric)
        self.index.set_graph(self.graph)

    def search_device(self, q_dev, k: int, ef: int, ids_dev, dists_dev, counters_dev, stream):
        """This shard's search; result slots past the pool are (0xffffffff, FLT_MAX)."""
        self.index.shard_search_device(q_dev.data_ptr(), q_dev.shape[0], k, ef, ids_dev.data_ptr(),
                                       dists_dev.data_ptr(), counters_dev.data_ptr(), stream)

    def search(self, q_dev, k: int, ef: int, stream, group=None):
        import torch

        nq = q_dev.shape[0]
        ids = torch.empty((nq, k), dtype=torch.int32, device=q_dev.device)
        d = torch.empty((nq, k), dtype=torch.float32, device=q_dev.device)
        c = torch.empty((nq, 4), dtype=torch.int32, device=q_dev.device)
        self.search_device(q_dev, k, ef, ids, d, c, stream)
        return exchange_and_merge(ids, d, self.lo, k, group)
