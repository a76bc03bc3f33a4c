"""Graph diagnostics of the device build at scale: recall / lost queries per build schedule,
level-0 in-degree, reachability of the ground-truth neighbours of lost queries."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--gen", default="text_like")
    ap.add_argument("--kw", default='{"latent": 16, "sigma_noise": 0.003}')
    ap.add_argument("--scheds", default="0,0,1;8192,0,1;0,64,1;0,0,2")
    ap.add_argument("--efs", default="200,800")
    a = ap.parse_args()
    import torch
    from alayalite_amd import _native
    import workloads.datasets as datasets

    ext = _native._ext
    metric = 1 if a.gen == "text_like" else 0
    base, q = getattr(datasets, a.gen)(a.n, 1000, **json.loads(a.kw))
    dev = torch.device("cuda", 0)
    gt = bench.exact_gt(torch, torch.from_numpy(base).to(dev), torch.from_numpy(q).to(dev), base, q, metric=metric)
    torch.cuda.empty_cache()
    ix = ext.DeviceIndex(0)
    ix.set_base(base, metric, None)
    for sched in a.scheds.split(";"):
        mb, bd, rf = (int(x) for x in sched.split(","))
        t = time.perf_counter()
        g, st = ix.build_graph(32, 100, 100, bd, mb, rf)
        bt = time.perf_counter() - t
        l0 = g.arrays()[0]
        indeg = np.bincount(l0[l0 != 0xFFFFFFFF].astype(np.int64), minlength=a.n)
        out = {"max_batch": mb, "batch_div": bd, "refine": rf, "build_s": round(bt, 1),
               "indeg0_frac": round(float(np.mean(indeg == 0)), 5)}
        for ef in (int(x) for x in a.efs.split(",")):
            ids, _, _ = ix.search(q, 10, ef)
            per_q = np.array([len(set(x.tolist()) & set(y.tolist())) for x, y in zip(ids, gt)])
            lost = np.nonzero(per_q == 0)[0]
            out[f"ef{ef}"] = {"recall": round(float(per_q.mean() / 10), 4), "lost": round(float(len(lost) / len(per_q)), 4),
                              "lost_gt_indeg0": round(float(np.mean(indeg[gt[lost]] == 0)), 4) if len(lost) else None,
                              "lost_gt_id_mean": round(float(gt[lost].mean()), 1) if len(lost) else None}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
