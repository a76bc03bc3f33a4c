"""One rank of the sharded-search GPU test (tests/test_shard_gpu.py), started as a child process.

Every rank runs on cuda:0 with a gloo group (a one-GPU box rehearses the N-GPU path; bench.py runs
the same ShardedIndex / exchange_and_merge code over RCCL).  The rank builds its shard's graph on
the host, searches the queries on the device (ShardedIndex.search: shard_search_device + the
all_gather exchange + merge, on device tensors), and writes the merged result plus the oracle's
search of its own shard (the restatement of search_solo on the shard's graph) for rank 0 to check.

argv: out_dir n dim nq k ef seed
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out_dir, n, dim, nq, k, ef, seed = sys.argv[1], *map(int, sys.argv[2:8])
    import torch
    import torch.distributed as dist

    import oracle
    from alayalite_amd import _native
    from alayalite_amd.sharded import EMPTY, ShardedIndex

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    rng = np.random.default_rng(seed)
    centres = rng.uniform(0, 0.5, (32, dim)).astype(np.float32)
    base = np.clip(centres[rng.integers(0, 32, n)] + rng.normal(0, 0.05, (n, dim)), 0, 1).astype(np.float32)
    queries = np.clip(centres[rng.integers(0, 32, nq)] + rng.normal(0, 0.05, (nq, dim)), 0, 1).astype(np.float32)

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    shard = ShardedIndex(base, world, rank, device=0, num_threads=4)
    q_dev = torch.from_numpy(queries).to(dev)
    stream = torch.cuda.current_stream(dev)
    ids, dists = shard.search(q_dev, k, ef, stream.cuda_stream)
    torch.cuda.synchronize()

    # the oracle's search of this shard (local ids); slots past the pool -> (EMPTY, FLT_MAX), the
    # shard search's fill (the restatement's LinearPool reads (0, 0.0) there, index.hpp:301)
    _native._ext  # noqa: B018  (the extension is loaded: the product path ran above)
    oracle.build()
    l0, levels, off, ue, ep, upper_r, _ = shard.graph.arrays()
    view = oracle.IndexView(shard.rows, l0, levels, off, ue, upper_r, ep)
    o_ids = np.zeros((nq, k), np.uint32)
    o_d = np.zeros((nq, k), np.float32)
    pool = min(ef, shard.rows.shape[0])
    for i in range(nq):
        o_ids[i], o_d[i] = view.search(queries[i], k, ef)
        o_ids[i, pool:] = EMPTY
        o_d[i, pool:] = np.finfo(np.float32).max
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), merged_ids=ids.cpu().numpy(), merged_d=dists.cpu().numpy(),
             shard_ids=o_ids, shard_d=o_d, lo=shard.lo)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
