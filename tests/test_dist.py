"""Multi-process shard exchange + merge on CPU (gloo, world_size 2): the same code path bench.py
runs over RCCL/xGMI, checked against a numpy restatement of the merge."""

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_results(rank, nq=37, k=10, n_per=500, seed=0):
    rng = np.random.default_rng(seed + rank)
    ids = np.stack([rng.choice(n_per, k, replace=False) for _ in range(nq)]).astype(np.int32)
    d = np.sort(rng.random((nq, k)).astype(np.float32), axis=1)
    d[:, 3] = d[:, 2]  # ties inside a shard
    if rank == 1:
        d[:5, 0] = _shard_results(0, nq, k, n_per, seed)[1][:5, 0]  # ties across shards
    return ids, d


def _with_empty_slots(rank, ids, d):
    """A shard search with fewer pool entries than k (shard rows < k or ef < k) fills the rest with
    (0xffffffff, FLT_MAX) (alaya_index_shard_search_device)."""
    if rank == 1:
        ids, d = ids.copy(), d.copy()
        ids[:, 4:] = -1  # int32 view of 0xffffffff
        d[:, 4:] = np.finfo(np.float32).max
        d[:3, :4] = 0.0  # shard 1's real candidates precede shard 0's for the first queries
    return ids, d


def _worker(rank, world, port, out_path, empty=False):
    import torch.distributed as dist

    from alayalite_amd.sharded import exchange_and_merge

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids, d = _shard_results(rank)
    if empty:
        ids, d = _with_empty_slots(rank, ids, d)
    mi, md = exchange_and_merge(torch.from_numpy(ids), torch.from_numpy(d), rank * 500, 10)
    if rank == 0:
        np.savez(out_path, ids=mi.numpy(), d=md.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_everything():
    from alayalite_amd.sharded import shard_range

    for n, w in [(1_000_000, 8), (10, 3), (7, 8), (1000, 1)]:
        spans = [shard_range(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_exchange_and_merge_gloo(tmp_path):
    import torch.multiprocessing as mp

    from alayalite_amd.sharded import merge_reference

    out = str(tmp_path / "merged.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    parts = [_shard_results(r) for r in range(2)]
    ref_i, ref_d = merge_reference([p[0] for p in parts], [p[1] for p in parts], [0, 500], 10)
    assert np.array_equal(got["ids"], ref_i)
    assert np.array_equal(got["d"], ref_d)


def test_exchange_with_empty_slots_gloo(tmp_path):
    """Empty slots never displace a real candidate (a (0, 0.0) fill became a spurious top
    hit); with fewer than k real candidates in all shards together the result ends in empty slots."""
    import torch.multiprocessing as mp

    from alayalite_amd.sharded import EMPTY, merge_reference

    out = str(tmp_path / "merged.npz")
    mp.spawn(_worker, args=(2, _free_port(), out, True), nprocs=2, join=True)
    got = np.load(out)
    parts = [_with_empty_slots(r, *_shard_results(r)) for r in range(2)]
    ref_i, ref_d = merge_reference([p[0] for p in parts], [p[1] for p in parts], [0, 500], 10)
    assert np.array_equal(got["ids"], ref_i) and np.array_equal(got["d"], ref_d)
    assert not (got["ids"] == EMPTY).any()  # shard 0 alone holds 10 real candidates per query
    assert (got["ids"][:3, :4] >= 500).all()  # shard 1's zero-distance rows come first
    # fewer than k real candidates overall: the merged tail is empty slots
    from alayalite_amd.sharded import pack_candidates, to_global, unpack_candidates

    a_i, a_d = np.full((2, 3), -1, np.int32), np.full((2, 3), np.finfo(np.float32).max, np.float32)
    a_i[:, 0], a_d[:, 0] = 7, 1.5
    keys = torch.cat([pack_candidates(to_global(torch.from_numpy(a_i), 0), torch.from_numpy(a_d)),
                      pack_candidates(to_global(torch.from_numpy(a_i), 100), torch.from_numpy(a_d))], 1)
    gi, gd = unpack_candidates(torch.sort(keys, 1).values[:, :4])
    assert gi[0].tolist() == [7, 107, EMPTY, EMPTY]


def test_packed_keys_order_like_dist_then_id():
    """The exchange packs (distance, global id) into one int64 whose order is (dist asc, id asc):
    negative distances (IP), -0.0 vs +0.0 and ties across ids included; the merge result equals the
    two-sort merge."""
    from alayalite_amd.sharded import merge_topk, pack_candidates, unpack_candidates

    rng = np.random.default_rng(3)
    d = np.concatenate([rng.normal(size=(40, 30)).astype(np.float32), np.zeros((40, 2), np.float32),
                        np.full((40, 2), -0.0, np.float32), np.full((40, 2), np.inf, np.float32)], 1)
    d[:, 4] = d[:, 7]
    ids = rng.integers(0, 2 ** 31 - 1, d.shape).astype(np.int64)
    dt, it = torch.from_numpy(d), torch.from_numpy(ids)
    gi, gd = unpack_candidates(torch.sort(pack_candidates(it, dt), 1).values[:, :10])
    mi, md = merge_topk(it, dt + 0.0, 10)
    assert torch.equal(gi, mi) and torch.equal(gd.view(torch.int32), (md + 0.0).view(torch.int32))


def _fake_shard(rank, n_per=300, d=8):
    return np.random.default_rng(100 + rank).random((n_per, d), dtype=np.float32)


def _fake_search(rank, k):
    """A stand-in shard search on CPU tensors: exact top-k of the batch against this rank's rows,
    (dist, id) order, written into the pipeline's buffers like shard_search_device would."""
    rows = _fake_shard(rank)

    def fn(q, ids, d, c, stream):
        qa = q.numpy()
        dd = ((qa[:, None, :] - rows[None, :, :]) ** 2).sum(-1).astype(np.float32)
        o = np.stack([np.lexsort((np.arange(rows.shape[0]), r))[:k] for r in dd])
        ids.copy_(torch.from_numpy(o.astype(np.int32)))
        d.copy_(torch.from_numpy(np.take_along_axis(dd, o, 1)))
        c.zero_()

    return fn


def _pipeline_worker(rank, world, port, out_path):
    import torch.distributed as dist

    from alayalite_amd.sharded import ShardPipeline

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    batches = [torch.from_numpy(rng.random((23, 8), dtype=np.float32)) for _ in range(5)]
    with ShardPipeline(_fake_search(rank, 10), 23, 10, rank * 300, "cpu") as pipe:  # (close() on exit)
        over = pipe.run(batches)
        sync = pipe.run_sync(batches)
    if rank == 0:
        np.savez(out_path, over_i=np.stack([o[0].numpy() for o in over]), over_d=np.stack([o[1].numpy() for o in over]),
                 sync_i=np.stack([o[0].numpy() for o in sync]), sync_d=np.stack([o[1].numpy() for o in sync]),
                 q=np.stack([b.numpy() for b in batches]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_pipeline_gloo(tmp_path):
    """ShardPipeline (double-buffered batches: search i+1 issued before exchange i) returns, batch
    for batch, what the synchronous loop and the numpy merge restatement return."""
    import torch.multiprocessing as mp

    from alayalite_amd.sharded import merge_reference

    out = str(tmp_path / "pipe.npz")
    mp.spawn(_pipeline_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    assert np.array_equal(got["over_i"], got["sync_i"]) and np.array_equal(got["over_d"], got["sync_d"])
    for b in range(got["q"].shape[0]):
        parts = []
        for r in range(2):
            ids = torch.empty((23, 10), dtype=torch.int32)
            d = torch.empty((23, 10), dtype=torch.float32)
            _fake_search(r, 10)(torch.from_numpy(got["q"][b]), ids, d, torch.empty((23, 4), dtype=torch.int32), 0)
            parts.append((ids.numpy(), d.numpy()))
        ref_i, ref_d = merge_reference([p[0] for p in parts], [p[1] for p in parts], [0, 300], 10)
        assert np.array_equal(got["over_i"][b], ref_i) and np.array_equal(got["over_d"][b], ref_d)


def _layout_worker(rank, world, port, out_path, shards):
    """S shards x (world / S) query groups: rank r searches its group's query slice on its shard
    (exact top-k stand-in), the group's ranks exchange inside their own process group, and every
    group's merged rows are gathered back into query order."""
    import torch.distributed as dist

    from alayalite_amd.sharded import Layout, exchange_and_merge, gather_layout_results

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lay = Layout(world, rank, shards)
    group = lay.new_groups(dist)
    base, queries = _layout_data()
    lo, hi = lay.rows(base.shape[0])
    qa, qb = lay.queries(queries.shape[0])
    rows = base[lo:hi]
    q = queries[qa:qb]
    dd = ((q[:, None, :] - rows[None, :, :]) ** 2).sum(-1).astype(np.float32)
    o = np.stack([np.lexsort((np.arange(rows.shape[0]), r))[:10] for r in dd])
    ids, d = torch.from_numpy(o.astype(np.int32)), torch.from_numpy(np.take_along_axis(dd, o, 1))
    mi, md = exchange_and_merge(ids, d, lo, 10, group)
    gi, gd = gather_layout_results(mi, md, lay, queries.shape[0], dist)
    if rank == 0:
        np.savez(out_path, ids=gi.numpy(), d=gd.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _layout_data():
    rng = np.random.default_rng(11)
    return rng.random((601, 6), dtype=np.float32), rng.random((29, 6), dtype=np.float32)


@pytest.mark.parametrize("shards", [2, 1, 4])
def test_shards_by_query_groups_gloo(tmp_path, shards):
    """world 4 as 2 shards x 2 query groups (and 1 x 4, 4 x 1): the merged result of every query
    equals merge_reference over the per-shard exact top-k, and -- the stand-in search being exact --
    the exact top-k of the whole base by (distance, id)."""
    import torch.multiprocessing as mp

    from alayalite_amd.sharded import merge_reference, shard_range

    out = str(tmp_path / "layout.npz")
    mp.spawn(_layout_worker, args=(4, _free_port(), out, shards), nprocs=4, join=True)
    got = np.load(out)
    base, queries = _layout_data()
    parts, offs = [], []
    for s in range(shards):
        lo, hi = shard_range(base.shape[0], shards, s)
        dd = ((queries[:, None, :] - base[None, lo:hi, :]) ** 2).sum(-1).astype(np.float32)
        o = np.stack([np.lexsort((np.arange(hi - lo), r))[:10] for r in dd])
        parts.append((o.astype(np.int32), np.take_along_axis(dd, o, 1)))
        offs.append(lo)
    ref_i, ref_d = merge_reference([p[0] for p in parts], [p[1] for p in parts], offs, 10)
    assert np.array_equal(got["ids"], ref_i) and np.array_equal(got["d"], ref_d)
    full = ((queries[:, None, :] - base[None, :, :]) ** 2).sum(-1).astype(np.float32)
    exact = np.stack([np.lexsort((np.arange(base.shape[0]), r))[:10] for r in full])
    assert np.array_equal(got["ids"], exact)


def test_layout_rank_map():
    from alayalite_amd.sharded import Layout

    lays = [Layout(8, r, 2) for r in range(8)]
    assert [(x.shard, x.group) for x in lays] == [(r % 2, r // 2) for r in range(8)]
    assert lays[5].group_ranks == [4, 5] and lays[5].queries(10000) == (5000, 7500)
    assert Layout(8, 3, 8).queries(10000) == (0, 10000) and Layout(8, 3, 1).rows(100) == (0, 100)
    with pytest.raises(ValueError):
        Layout(8, 0, 3)
