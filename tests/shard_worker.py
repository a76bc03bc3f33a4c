"""One rank of the sharded-search GPU test (tests/test_shard_gpu.py), started as a child process.

Every rank runs on cuda:0 with a gloo group (a one-GPU box rehearses the N-GPU path; bench.py runs
the same ShardedIndex / exchange_and_merge code over RCCL), or, with ALAYA_TEST_BACKEND=nccl, as a
single rank over RCCL itself.  The rank builds its shard's graph on
the host, searches the queries on the device (ShardedIndex.search: shard_search_device + the
all_gather exchange + merge, on device tensors), and writes the merged result plus the oracle's
search of its own shard (the restatement of search_solo on the shard's graph) for rank 0 to check.

mode "sq8" (config 5's path): 768-d-style unit-sphere rows, IP, each shard with its own SQ8 space;
the shard search is the SQ8 graph search plus PyIndex::rerank, whose id-0 entries belong to the
shard holding global row 0 (alaya_index_shard_search_sq8_device); the oracle side is the
restatement's SQ8 search of the shard plus its rerank (ef - k zero entries only on that shard).
Both modes also run the queries through ShardPipeline (double-buffered batches, search i+1 beside
exchange i) and save that result too.

argv: out_dir n dim nq k ef seed [mode: f32 | sq8]
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _data(mode, n, dim, nq, seed):
    rng = np.random.default_rng(seed)
    if mode == "sq8":  # text-embedding-shaped: clusters on the unit sphere, rows normalised
        centres = rng.standard_normal((16, dim)).astype(np.float32)
        centres /= np.linalg.norm(centres, axis=1, keepdims=True)

        def draw(m):
            x = centres[rng.integers(0, 16, m)] + rng.normal(0, 0.03, (m, dim)).astype(np.float32)
            return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)

        base, queries = draw(n), draw(nq)
        # two queries next to shard-local row 0 of each shard: global row 0's id-0 entries are the
        # reference's quirk and may repeat; the other shard's local row 0 must not
        lo1 = (n + 1) // 2
        queries[0] = base[0] * 0.999 + 0.001 * queries[0]
        queries[1] = base[lo1] * 0.999 + 0.001 * queries[1]
        return base, queries
    centres = rng.uniform(0, 0.5, (32, dim)).astype(np.float32)
    base = np.clip(centres[rng.integers(0, 32, n)] + rng.normal(0, 0.05, (n, dim)), 0, 1).astype(np.float32)
    queries = np.clip(centres[rng.integers(0, 32, nq)] + rng.normal(0, 0.05, (nq, dim)), 0, 1).astype(np.float32)
    return base, queries


def main():
    out_dir, n, dim, nq, k, ef, seed = sys.argv[1], *map(int, sys.argv[2:8])
    mode = sys.argv[8] if len(sys.argv) > 8 else "f32"
    import torch
    import torch.distributed as dist

    import oracle
    from alayalite_amd import _native
    from alayalite_amd.sharded import EMPTY, ShardedIndex

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # ALAYA_TEST_BACKEND=nccl: RCCL on cuda:0 (one rank per GPU -- a one-GPU box runs world 1), the
    # device-tensor all_gather bench.py uses on a node; default gloo (several ranks on one GPU)
    if os.environ.get("ALAYA_TEST_BACKEND", "gloo") == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo")
    base, queries = _data(mode, n, dim, nq, seed)
    metric = 1 if mode == "sq8" else 0

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    shard = ShardedIndex(base, world, rank, device=0, metric=metric, num_threads=4, sq8=(mode == "sq8"))
    q_dev = torch.from_numpy(queries).to(dev)
    stream = torch.cuda.current_stream(dev)
    ids, dists = shard.search(q_dev, k, ef, stream.cuda_stream)
    torch.cuda.synchronize()
    # the same queries in three batches through the double-buffered pipeline
    cuts = [0, nq // 3, 2 * nq // 3, nq]
    batches = [q_dev[cuts[i]:cuts[i + 1]].contiguous() for i in range(3)]
    # ALAYA_TEST_RESERVE_CUS: the pipeline's search on a CU-masked stream that leaves CUs to the exchange
    pipe = shard.pipeline(max(b.shape[0] for b in batches), k, ef,
                          reserve_cus=int(os.environ.get("ALAYA_TEST_RESERVE_CUS", "0")))
    res = pipe.run(batches)
    torch.cuda.synchronize()
    pipe.close()
    pipe_ids = [r[0].cpu().numpy() for r in res]
    pipe_d = [r[1].cpu().numpy() for r in res]

    # the oracle's search (+ rerank) of this shard, local ids; empty slots -> (EMPTY, FLT_MAX), the
    # shard search's fill (the restatement's LinearPool reads (0, 0.0) there, index.hpp:301)
    _native._ext  # noqa: B018  (the extension is loaded: the product path ran above)
    oracle.build()
    l0, levels, off, ue, ep, upper_r, _ = shard.graph.arrays()
    view = oracle.IndexView(shard.rows, l0, levels, off, ue, upper_r, ep, metric=metric,
                            sq8=shard.sq8 if mode == "sq8" else None)
    o_ids = np.zeros((nq, k), np.uint32)
    o_d = np.zeros((nq, k), np.float32)
    pool = min(ef, shard.rows.shape[0])
    for i in range(nq):
        s_ids, s_d = view.search(queries[i], k, ef)
        if mode == "sq8":
            assert pool >= k, "the sq8 worker needs full pools"
            # PyIndex::rerank (index.hpp:450-488): the ef - k zero entries only where row 0 is global
            # row 0; elsewhere the k search ids alone (ef = k: no zero entries)
            s_ids, s_d = view.rerank(queries[i], s_ids, k, ef if shard.lo == 0 else k)
        else:
            s_ids[pool:] = EMPTY
            s_d[pool:] = np.finfo(np.float32).max
        o_ids[i], o_d[i] = s_ids, s_d
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), merged_ids=ids.cpu().numpy(), merged_d=dists.cpu().numpy(),
             pipe_ids=np.concatenate(pipe_ids), pipe_d=np.concatenate(pipe_d),
             shard_ids=o_ids, shard_d=o_d, lo=shard.lo)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
