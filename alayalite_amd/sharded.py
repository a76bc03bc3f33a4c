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


class Layout:
    """S range shards x G = world / S query groups over `world` ranks (S divides world).

    Rank r holds shard s = r % S (rows shard_range(n, S, s)) and answers query group g = r // S
    (queries shard_range(nq, G, g)); the S ranks of a group -- g*S .. g*S + S - 1, neighbours on one
    node -- exchange their per-shard top-k inside their own process group.  S = world is the
    north star's pure base-range sharding (every rank sees every query), S = 1 pure query
    splitting over whole-index replicas (no collective on the data path).  Each of the S shards is
    held by G ranks; total work per step is fixed ("strong")."""

    def __init__(self, world: int, rank: int, shards: int):
        if shards < 1 or world % shards:
            raise ValueError(f"shards ({shards}) must divide the number of ranks ({world})")
        self.world, self.rank, self.shards = world, rank, shards
        self.groups = world // shards
        self.shard, self.group = rank % shards, rank // shards
        self.group_ranks = list(range(self.group * shards, (self.group + 1) * shards))

    def rows(self, n: int) -> tuple[int, int]:
        return shard_range(n, self.shards, self.shard)

    def queries(self, nq: int) -> tuple[int, int]:
        return shard_range(nq, self.groups, self.group)

    def new_groups(self, dist):
        """Create every query group's process group (collective: every rank calls it, in the same
        order) and return this rank's -- None when a group is the whole world (use the default)."""
        if self.groups == 1:
            return None
        mine = None
        for g in range(self.groups):
            pg = dist.new_group(list(range(g * self.shards, (g + 1) * self.shards)))
            if g == self.group:
                mine = pg
        return mine


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

    return exchange_packed(pack_candidates(to_global(local_ids, offset), local_dists), k, group)


def exchange_packed(packed, k: int, group=None):
    """The exchange of already packed keys (pack_candidates of global ids): one all_gather and the
    merge sort; returns (ids, dists) on the keys' device.  With gloo on device tensors the keys go
    through the host (copies only -- no device kernels between the copies)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    device = packed.device
    if world == 1:  # a one-shard layout (S = 1): nothing to exchange, the sort gives the (dist, id) order
        best = torch.sort(packed, dim=1).values[:, :k]
        ids, d = unpack_candidates(best)
        return ids, d
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


def shard_search(index, lo: int, sq8: bool, q_dev, k: int, ef: int, ids_dev, dists_dev, counters_dev, stream,
                 rq_dev=None):
    """One shard's search of a device query batch into device buffers (asynchronous on `stream`, a
    hipStream_t handle); result slots without a candidate are (0xffffffff, FLT_MAX).  SQ8 shards run
    the SQ8 graph search plus PyIndex::rerank (index.hpp:337-345, 450-488); the reference's id-0
    entries belong to global row 0, i.e. to the shard with lo == 0 (rq_dev: the rerank queries,
    None = q_dev)."""
    nq = q_dev.shape[0]
    if sq8:
        index.shard_search_sq8_device(q_dev.data_ptr(), 0 if rq_dev is None else rq_dev.data_ptr(), nq, k, ef,
                                      lo == 0, ids_dev.data_ptr(), dists_dev.data_ptr(), counters_dev.data_ptr(),
                                      stream)
    else:
        index.shard_search_device(q_dev.data_ptr(), nq, k, ef, ids_dev.data_ptr(), dists_dev.data_ptr(),
                                  counters_dev.data_ptr(), stream)


class ShardPipeline:
    """Double-buffered query batches (overlap the exchange with the next batch's search).

    Batch i's search runs on the compute stream into buffer slot i % 2, followed there by the packing
    of its (distance, global id) keys (a few elementwise kernels); its exchange (one all_gather, the
    merge sort) runs on a second stream once the packing's event fires, while the compute stream
    already searches batch i + 1.  Packing on the compute stream matters: the search kernel is
    persistent and holds every CU slot it can, so a kernel queued on another stream behind it waits
    for it to drain -- with gloo the exchange stream then carries only copies.  The exchange reads
    only the packed keys, so slot i % 2's buffers are free for batch i + 2 once the compute stream
    has packed them (stream order).  The host issues
    search i + 1 before exchange i, so a blocking exchange (gloo with host copies) still overlaps the
    device search.  On CPU tensors (gloo tests) the same loop runs without streams.

    search_fn(q, ids, dists, counters, stream_handle) launches one shard search (shard_search);
    batches hold at most nq queries each.

    reserve_cus > 0 runs the compute stream on a CU-masked stream that leaves that many CUs to other
    streams (alaya_stream_create_reserving): the search sizes its persistent grid to the CUs left,
    so the exchange's kernels (RCCL's all_gather and the merge sort) start at once instead of
    queueing behind the next batch's search."""

    def __init__(self, search_fn, nq: int, k: int, offset: int, device, group=None, timing: bool = False,
                 reserve_cus: int = 0):
        import torch

        self.search_fn, self.k, self.offset, self.group = search_fn, k, offset, group
        self.device = torch.device(device)
        mk = lambda dt, w: torch.empty((nq, w), dtype=dt, device=self.device)  # noqa: E731
        self.bufs = [(mk(torch.int32, k), mk(torch.float32, k), mk(torch.int32, 4)) for _ in range(2)]
        self.rows = [0, 0]
        self.packed = [None, None]  # packed keys of the batch in each slot (compute stream)
        self.gpu = self.device.type == "cuda"
        self._masked = None
        self.closed = False
        if self.gpu:
            if reserve_cus > 0:
                from ._native import _ext

                self._masked = _ext.stream_create_reserving(self.device.index or 0, int(reserve_cus))
                self.compute = torch.cuda.ExternalStream(self._masked, device=self.device)
            else:
                self.compute = torch.cuda.Stream(self.device)
            self.exch = torch.cuda.Stream(self.device)
            self.searched = [torch.cuda.Event() for _ in range(2)]
        self.timing = timing and self.gpu
        self.spans = []  # (start, end) events around each search on the compute stream (timing=True)

    def _slot(self, slot, m):
        """Buffers of slot for a batch of m <= nq queries (leading rows: contiguous views)."""
        return tuple(b[:m] for b in self.bufs[slot])

    def _launch(self, q, slot):
        ids, d, c = self._slot(slot, q.shape[0])
        self.rows[slot] = q.shape[0]
        if not self.gpu:
            self.search_fn(q, ids, d, c, 0)
            return
        import torch

        if self.timing:

            span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            span[0].record(self.compute)
        self.search_fn(q, ids, d, c, self.compute.cuda_stream)
        if self.timing:
            span[1].record(self.compute)
            self.spans.append(span)
        with torch.cuda.stream(self.compute):
            self.packed[slot] = pack_candidates(to_global(ids, self.offset), d)
        self.searched[slot].record(self.compute)

    def _exchange(self, slot):
        import torch

        ids, d, _ = self._slot(slot, self.rows[slot])
        if not self.gpu:
            return exchange_and_merge(ids, d, self.offset, self.k, self.group)
        with torch.cuda.stream(self.exch):
            self.exch.wait_event(self.searched[slot])
            packed = self.packed[slot]
            packed.record_stream(self.exch)
            out = exchange_packed(packed, self.k, self.group)
        return out

    def run(self, batches):
        """Search + exchange every batch (device query tensors); returns the merged (ids, dists) per
        batch, produced on the exchange stream (synchronise before reading them on the host)."""
        if self.closed:
            raise RuntimeError("ShardPipeline used after close()")
        out = [None] * len(batches)
        if not batches:
            return out
        if self.gpu:  # the batches were produced on the caller's stream
            import torch

            self.compute.wait_stream(torch.cuda.current_stream(self.device))
        self._launch(batches[0], 0)
        for i in range(len(batches)):
            if i + 1 < len(batches):
                self._launch(batches[i + 1], (i + 1) % 2)
            out[i] = self._exchange(i % 2)
        if self.gpu:  # later work on the caller's stream sees the merged results
            import torch

            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.exch)
            for ids, d in out:  # allocated on the exchange stream, used on the caller's
                ids.record_stream(cur)
                d.record_stream(cur)
        return out

    def close(self):
        """Release the CU-masked compute stream (after the pipeline's work is done)."""
        if self._masked is not None:
            import torch

            from ._native import _ext

            torch.cuda.synchronize(self.device)
            _ext.stream_destroy(self._masked)
            self._masked = None
            self.compute = None  # the ExternalStream wrapped the freed handle
        self.closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def search_ms(self):
        """Mean search time (ms) of the batches run with timing=True, as the compute stream saw it
        inside the pipeline (after synchronisation)."""
        return float(np.mean([a.elapsed_time(b) for a, b in self.spans])) if self.spans else None

    def run_sync(self, batches):
        """The same batches without overlap: search, then exchange, one after the other on the
        caller's current stream (the synchronous reference for the overlapped timing)."""
        import torch

        out = []
        for q in batches:
            ids, d, c = self._slot(0, q.shape[0])
            stream = torch.cuda.current_stream(self.device).cuda_stream if self.gpu else 0
            self.search_fn(q, ids, d, c, stream)
            out.append(exchange_and_merge(ids, d, self.offset, self.k, self.group))
        return out


class ShardedIndex:
    """This rank's shard on its GPU: rows [lo, hi) of `base`, graph built on the shard.  sq8=True
    adds the shard's SQ8 space (SQ8Space::fit on the shard's rows, sq8_space.hpp:116-127): searches
    then run on the codes and rerank on the f32 rows (config 5)."""

    def __init__(self, base, world: int, rank: int, device: int = 0, metric: int = 0, R: int = 32,
                 ef_construction: int = 100, num_threads: int = 1, graph=None, sq8: bool = False):
        from ._native import _ext

        self.lo, self.hi = shard_range(base.shape[0], world, rank)
        self.rows = np.ascontiguousarray(base[self.lo:self.hi])
        self.graph = graph if graph is not None else _ext.Graph.build(self.rows, metric, R, ef_construction, num_threads, 100)
        self._device = device
        self.index = _ext.DeviceIndex(device)
        self.index.set_base(self.rows, metric)
        self.index.set_graph(self.graph)
        self.sq8 = None
        if sq8:
            mn, mx = _ext.sq8_train(self.rows)
            order = _ext.host_sq8_order()
            codes = _ext.sq8_encode(self.rows, mn, mx, max(1, num_threads))
            self.index.set_sq8(codes, mn, mx, order)
            self.sq8 = (codes, mn, mx, order)

    def search_device(self, q_dev, k: int, ef: int, ids_dev, dists_dev, counters_dev, stream, rq_dev=None):
        """This shard's search; result slots without a candidate are (0xffffffff, FLT_MAX)."""
        shard_search(self.index, self.lo, self.sq8 is not None, q_dev, k, ef, ids_dev, dists_dev, counters_dev,
                     stream, rq_dev)

    def search(self, q_dev, k: int, ef: int, stream, group=None):
        import torch

        nq = q_dev.shape[0]
        ids = torch.empty((nq, k), dtype=torch.int32, device=q_dev.device)
        d = torch.empty((nq, k), dtype=torch.float32, device=q_dev.device)
        c = torch.empty((nq, 4), dtype=torch.int32, device=q_dev.device)
        self.search_device(q_dev, k, ef, ids, d, c, stream)
        return exchange_and_merge(ids, d, self.lo, k, group)

    def pipeline(self, nq: int, k: int, ef: int, group=None, reserve_cus: int = 0) -> ShardPipeline:
        """A double-buffered pipeline for batches of nq queries at this ef (ShardPipeline)."""
        fn = lambda q, ids, d, c, s: self.search_device(q, k, ef, ids, d, c, s)  # noqa: E731
        return ShardPipeline(fn, nq, k, self.lo, self.index_device(), group, reserve_cus=reserve_cus)

    def index_device(self):
        import torch

        return torch.device("cuda", self._device)


def gather_layout_results(ids, dists, layout: Layout, nq: int, dist):
    """Every query group's merged (ids, dists) -> the whole batch in query order, on every rank
    (untimed: recall checks).  The ranks of a group hold the same merged rows; group g's rows come
    from its first rank.  Slices are padded to ceil(nq / G) rows for the all_gather."""
    import torch

    per = (nq + layout.groups - 1) // layout.groups
    dev = ids.device
    if dist.get_backend() == "gloo" and dev.type != "cpu":
        ids, dists = ids.cpu(), dists.cpu()
    pi = torch.zeros((per, ids.shape[1]), dtype=torch.int64, device=ids.device)
    pd = torch.zeros((per, ids.shape[1]), dtype=torch.float32, device=ids.device)
    pi[:ids.shape[0]] = ids.to(torch.int64)
    pd[:ids.shape[0]] = dists
    gi = [torch.empty_like(pi) for _ in range(layout.world)]
    gd = [torch.empty_like(pd) for _ in range(layout.world)]
    dist.all_gather(gi, pi)
    dist.all_gather(gd, pd)
    out_i, out_d = [], []
    for g in range(layout.groups):
        a, b = shard_range(nq, layout.groups, g)
        out_i.append(gi[g * layout.shards][:b - a])
        out_d.append(gd[g * layout.shards][:b - a])
    return torch.cat(out_i).to(dev), torch.cat(out_d).to(dev)
