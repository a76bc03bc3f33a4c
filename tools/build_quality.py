"""Device HNSW build vs host build: wall time and the recall@10 / QPS curve of each graph.

python tools/build_quality.py --gen gist_like --n 1000000 --nq 1000 [--host] [--batch-div 16 --max-batch 65536]
Prints one JSON line per builder: build seconds, device stats, and per-ef (recall, kernel ms)."""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (exact_gt, recall, host_threads)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", default="gist_like")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--efc", type=int, default=100)
    ap.add_argument("--batch-div", type=int, default=0)
    ap.add_argument("--max-batch", type=int, default=0)
    ap.add_argument("--refine", type=int, default=2)  # the library default (Index.fit(builder="gpu"))
    ap.add_argument("--variants", default="", help="extra device builds: 'efc:div:refine;...'")
    ap.add_argument("--host", action="store_true", help="also build on the host (16 threads) for comparison")
    ap.add_argument("--efs", default="40,80,120,200,300,400")
    a = ap.parse_args()
    import torch

    from alayalite_amd import _native
    import workloads.datasets as datasets

    native = _native._ext
    gen = getattr(datasets, a.gen)
    base, queries = gen(a.n, a.nq, a.dim) if a.dim else gen(a.n, a.nq)
    metric = 1 if a.gen == "text_like" else 0
    dev = torch.device("cuda", 0)
    bd = torch.from_numpy(base).to(dev)
    qd = torch.from_numpy(queries).to(dev)
    gt = bench.exact_gt(torch, bd, qd, base, queries, metric=metric)
    del bd
    torch.cuda.empty_cache()
    efs = [int(x) for x in a.efs.split(",")]

    def curve(ix):
        out = []
        for ef in efs:
            ix.search(queries, 10, ef)
            t = time.perf_counter()
            ids, _, cnt = ix.search(queries, 10, ef)
            ms = (time.perf_counter() - t) * 1e3
            out.append({"ef": ef, "recall": round(bench.recall(ids, gt), 4), "ms": round(ms, 3),
                        "n_dist": round(float(cnt[:, 0].mean()), 1)})
        return out

    ix = native.DeviceIndex(0)
    ix.set_base(base, metric, None)
    t = time.perf_counter()
    g, st = ix.build_graph(32, a.efc, 100, a.batch_div, a.max_batch, a.refine)
    wall = time.perf_counter() - t
    print(json.dumps({"builder": "gpu", "n": a.n, "gen": a.gen, "build_s": round(wall, 3), "stats": st,
                      "curve": curve(ix)}), flush=True)
    for v in filter(None, a.variants.split(";")):
        efc, bd, rf = (int(x) for x in v.split(":"))
        t = time.perf_counter()
        ix.build_graph(32, efc, 100, bd, 0, rf)
        wall = time.perf_counter() - t
        print(json.dumps({"builder": f"gpu efc{efc} div{bd} refine{rf}", "n": a.n, "build_s": round(wall, 3),
                          "curve": curve(ix)}), flush=True)
    if a.host:
        t = time.perf_counter()
        hg = native.Graph.build(base, metric, 32, a.efc, bench.host_threads(), 100)
        wall = time.perf_counter() - t
        hx = native.DeviceIndex(0)
        hx.set_base(base, metric, None)
        hx.set_graph(hg)
        print(json.dumps({"builder": "host", "threads": bench.host_threads(), "n": a.n, "gen": a.gen,
                          "build_s": round(wall, 3), "curve": curve(hx)}), flush=True)


if __name__ == "__main__":
    main()
