"""One-GPU rehearsal of bench.py --mode shard at G = 1, 2, 4, 8 (8-GPU runs are the driver's).

For each G: build the G base-range shard graphs on the device exactly as bench.py's ranks do
(alaya_index_build_graph, deterministic), search
every shard on this GPU in turn, merge the per-shard top-k by (dist, global id) with the same
merge the ranks use, pick the smallest ef of the sweep whose merged recall@10 >= 0.95, and time
each shard's kernel at that ef.  Predicted G-GPU QPS = nq / max over shards of the kernel time
(the all-gather of nq*k*8 B per rank and the merge are measured separately by bench.py).

usage: python tools/shard_rehearsal.py [--n 1000000] [--nq 10000] [--gs 1,2,4,8]   (config 4: 10k queries)
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=960)
    ap.add_argument("--gs", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    import bench as b
    from alayalite_amd import _native
    from alayalite_amd.sharded import merge_reference, shard_range
    from workloads.datasets import gist_like

    ext = _native._ext
    dev = torch.device("cuda", 0)
    base, queries = gist_like(args.n, args.nq, args.dim)
    q_dev = torch.from_numpy(queries).to(dev)
    gt, _ = b.exact_gt_flat(ext, base, queries, 0)
    torch.cuda.empty_cache()
    nq, K = args.nq, b.K
    results = []
    for G in [int(x) for x in args.gs.split(",")]:
        shards = []
        for r in range(G):
            lo, hi = shard_range(args.n, G, r)
            sb = np.ascontiguousarray(base[lo:hi])
            ix = ext.DeviceIndex(0)
            ix.set_base(sb, 0)
            t = time.time()
            ix.build_graph(b.R, 100, 100, 0, 0, 2)
            shards.append((lo, ix))
            print(f"G={G} shard {r}: rows [{lo},{hi}) device graph {time.time() - t:.1f}s", flush=True)
        ids = torch.empty((nq, K), dtype=torch.int32, device=dev)
        dd = torch.empty((nq, K), dtype=torch.float32, device=dev)
        cnt = torch.empty((nq, 4), dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev)

        def search_all(ef, timed=False):
            per_ids, per_d, times = [], [], []
            for lo, ix in shards:
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                ix.shard_search_device(q_dev.data_ptr(), nq, K, ef, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                       stream.cuda_stream)
                e.record(stream)
                torch.cuda.synchronize()
                times.append(a.elapsed_time(e))
                per_ids.append(ids.cpu().numpy().astype(np.int64))
                per_d.append(dd.cpu().numpy().copy())
            return per_ids, per_d, times

        sweep = []

        def probe(ef):
            per_ids, per_d, _ = search_all(ef)
            mi, _ = merge_reference(per_ids, per_d, [lo for lo, _ in shards], K)
            r = b.recall(mi, gt)
            sweep.append({"ef": ef, "recall": round(r, 4)})
            return r >= 0.95

        chosen = b.choose_ef(probe)
        search_all(chosen)  # warm
        worst = []
        for _ in range(args.steps):
            _, _, times = search_all(chosen)
            worst.append(max(times))
        ms = float(np.median(worst))
        row = {"G": G, "ef": chosen, "recall": next(x["recall"] for x in sweep if x["ef"] == chosen), "max_shard_kernel_ms": round(ms, 3),
               "predicted_qps": round(nq / (ms * 1e-3), 1), "sweep": sweep}
        results.append(row)
        print(json.dumps(row), flush=True)
        del shards
        torch.cuda.empty_cache()
    base_qps = results[0]["predicted_qps"]
    for r in results:
        r["predicted_efficiency"] = round(r["predicted_qps"] / (r["G"] * base_qps), 3)
    print(json.dumps(results))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
