"""Recall of device-built graphs across batch schedules vs the host builder (diagnostic)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    from alayalite_amd import _native
    import workloads.datasets as datasets

    native = _native._ext
    cases = [("uniform20k", lambda: datasets.uniform(20000, 200, 64, 3, 4), [16, 32, 64]),
             ("gist200k", lambda: datasets.gist_like(200000, 500), [40, 80, 160])]
    scheds = [(1, 1, 0), (64, 0, 0), (16, 0, 0), (64, 0, 1), (16, 0, 1), (8, 0, 1), (4, 0, 1)]
    for name, mk, efs in cases:
        base, q = mk()
        dev = torch.device("cuda", 0)
        gt = bench.exact_gt(torch, torch.from_numpy(base).to(dev), torch.from_numpy(q).to(dev), base, q)

        def curve(ix):
            return [round(bench.recall(ix.search(q, 10, ef)[0], gt), 4) for ef in efs]

        for th in (1, 16) if base.shape[0] <= 20000 else (16,):
            t = time.perf_counter()
            g = native.Graph.build(base, 0, 32, 100, th, 100)
            dt = time.perf_counter() - t
            ix = native.DeviceIndex(0)
            ix.set_base(base, 0, None)
            ix.set_graph(g)
            print(json.dumps({"case": name, "builder": f"host{th}", "s": round(dt, 2), "efs": efs,
                              "recall": curve(ix)}), flush=True)
        for bd, mb, rf in scheds:
            if mb == 1 and base.shape[0] > 20000:
                continue
            ix = native.DeviceIndex(0)
            ix.set_base(base, 0, None)
            t = time.perf_counter()
            _, st = ix.build_graph(32, 100, 100, bd, mb, rf)
            dt = time.perf_counter() - t
            print(json.dumps({"case": name, "builder": f"gpu div{bd} max{mb} refine{rf}", "s": round(dt, 2), "efs": efs,
                              "recall": curve(ix), "stats": st}), flush=True)


if __name__ == "__main__":
    main()
