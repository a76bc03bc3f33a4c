"""Recall@10 against ef for one graph of the headline workload (GIST-shaped 1M x 960, 1k queries,
workloads.datasets.gist_like -- bench.py's data), so the graphs the engine can search are compared
on the same rows, queries and exact ground truth:

  host1   the host builder on ONE thread: hnswlib add_point in label order, the reference's
          sequential insertion (hnswlib.hpp:652-751, seed 100); equal edge for edge to the oracle's
          builder (tests/test_builder.py).  Searched on the CPU with the oracle's coroutine batch
          driver (the reference's search restated; the device returns the same ids, tests/).
  device  the batched device build bench.py uses (alaya_index_build_graph, 2 refine passes),
          searched on the MI355X.

Ground truth: the exact top-10 (host1: oracle find_exact_gt restated, all cores; device: the
engine's exact flat path).  usage:
  python tools/graph_quality.py --graph host1 --out profiles/r06/graph_quality_host1.json   (CPU)
  python tools/graph_quality.py --graph device --out gpurun_out/graph_quality_device.json  (GPU)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

EFS = (60, 100, 150, 200, 250, 300, 350, 373, 387, 400, 450, 500, 600)


def recall(ids, gt):
    return float(np.mean([len(set(a[:10].tolist()) & set(b[:10].tolist())) / 10.0 for a, b in zip(ids, gt)]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", choices=("host1", "device"), required=True)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--out", required=True)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import workloads.datasets as ds

    t = time.time()
    base, queries = ds.gist_like(args.n, args.nq)
    print(f"data {base.shape} + {queries.shape} in {time.time() - t:.1f}s", flush=True)
    threads = args.threads or os.cpu_count()
    out = {"workload": f"gist_like {args.n} x {base.shape[1]}, {args.nq} queries (bench.py's headline data)",
           "graph": args.graph, "R": 32, "ef_construction": 100, "seed": 100, "curve": []}
    from alayalite_amd import _native

    ext = _native._ext
    if args.graph == "host1":
        import oracle

        oracle.build()
        t = time.time()
        gt, _ = oracle.exact_gt(base, queries, 10, threads)
        print(f"exact ground truth in {time.time() - t:.1f}s", flush=True)
        t = time.time()
        g = ext.Graph.build(base, 0, 32, 100, 1, 100)
        out["build_s"] = round(time.time() - t, 1)
        out["builder"] = "host, 1 thread (the reference's sequential insertion order)"
        print(f"graph (1 thread) in {out['build_s']}s", flush=True)
        l0, levels, off, ue, ep, ur, _ = g.arrays()
        view = oracle.IndexView(base, l0, levels, off, ue, ur, ep, metric=oracle.L2)
        for ef in EFS:
            ids, _, cnt, sec = view.batch_search(queries, 10, ef, threads)
            out["curve"].append({"ef": ef, "recall": round(recall(ids, gt), 4),
                                 "mean_n_dist": round(float(cnt[:, 0].mean()), 1)})
            print(out["curve"][-1], flush=True)
        out["search"] = f"oracle coroutine batch driver on {threads} host threads"
    else:
        import torch

        torch.cuda.is_available()
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        gt, _, _ = dev.flat_search(queries, 10)
        t = time.time()
        g, stats = dev.build_graph(32, 100, 100, 0, 0, 2)
        out["build_s"] = round(time.time() - t, 1)
        out["builder"] = "device, batched insertion + 2 refine passes (bench.py's default)"
        print(f"graph (device) in {out['build_s']}s", flush=True)
        for ef in EFS:
            ids, _, cnt = dev.search(queries, 10, ef)
            out["curve"].append({"ef": ef, "recall": round(recall(ids, gt), 4),
                                 "mean_n_dist": round(float(cnt[:, 0].mean()), 1)})
            print(out["curve"][-1], flush=True)
        out["search"] = "MI355X search kernel"
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
