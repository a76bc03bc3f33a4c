"""The shard exchange beside the persistent search, on one GPU over RCCL (one rank: a one-GPU box
holds one RCCL rank; bench.py runs the same ShardPipeline on a node).

For each CU reservation R (the pipeline's compute stream leaves R CUs to other streams,
alaya_stream_create_reserving, and the search sizes its grid to the CUs left) it times, on a
device-built graph and batches of --nq queries:
  * search alone: the shard search of each batch on the compute stream (events);
  * exchange alone: pack + RCCL all_gather + merge sort of a batch's results;
  * pipelined: ShardPipeline.run over --steps batches (search i+1 beside exchange i), wall clock.
overlapped / max(search, exchange) near 1 means the exchange is hidden.  JSON to --out.

usage: python tools/rccl_overlap.py [--workload gist|sift] [--nq 10000] [--steps 10] [--reserve 0,8]
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("gist", "sift"), default="gist")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=10000)
    ap.add_argument("--ef", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reserve", default="0,8")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    import torch
    import torch.distributed as dist

    from alayalite_amd import _native
    from alayalite_amd.sharded import ShardPipeline, exchange_and_merge, shard_search
    import workloads.datasets as ds

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    ext = _native._ext
    dim, ef = (960, args.ef or 373) if args.workload == "gist" else (128, args.ef or 70)
    gen = ds.gist_like if args.workload == "gist" else ds.sift_like
    base, queries = gen(args.n, args.nq, dim)
    index = ext.DeviceIndex(0)
    index.set_base(base, 0)
    index.build_graph(32, 100, 100, 0, 0, 2)
    del base
    q = torch.from_numpy(np.ascontiguousarray(queries)).to(dev)
    K = 10
    fn = lambda qq, i, d, c, s: shard_search(index, 0, False, qq, K, ef, i, d, c, s)  # noqa: E731
    rows = []
    for reserve in [int(x) for x in args.reserve.split(",")]:
        # search alone, on the (masked) compute stream of a pipeline
        tp = ShardPipeline(fn, args.nq, K, 0, dev, timing=True, reserve_cus=reserve)
        ids, dd, cc = tp._slot(0, args.nq)
        st = tp.compute
        fn(q, ids, dd, cc, st.cuda_stream)
        torch.cuda.synchronize()
        g, w = index.last_launch()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        for a, b_ in ev:
            a.record(st)
            fn(q, ids, dd, cc, st.cuda_stream)
            b_.record(st)
        torch.cuda.synchronize()
        search_ms = float(np.median([a.elapsed_time(b_) for a, b_ in ev]))
        # exchange alone
        exchange_and_merge(ids, dd, 0, K)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            exchange_and_merge(ids, dd, 0, K)
        torch.cuda.synchronize()
        exch_ms = (time.perf_counter() - t0) / args.steps * 1e3
        # pipelined
        tp.run([q] * 2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp.run([q] * args.steps)
        torch.cuda.synchronize()
        pipe_ms = (time.perf_counter() - t0) / args.steps * 1e3
        tp.close()
        row = {"reserved_cus": reserve, "searchers": int(g) * int(w), "search_ms": round(search_ms, 4),
               "exchange_ms": round(exch_ms, 4), "overlapped_ms_per_step": round(pipe_ms, 4),
               "overlapped_over_max": round(pipe_ms / max(search_ms, exch_ms), 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"workload": args.workload, "n": args.n, "nq": args.nq, "ef": ef, "steps": args.steps, "rows": rows,
           "note": "one rank over RCCL (world size 1): the all_gather is a local copy here, so this shows the "
                   "stream and grid mechanics and the search's cost of the reservation, not xGMI traffic"}
    print(json.dumps(out), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
