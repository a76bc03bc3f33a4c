"""Recall diagnostic for the config-5-shaped workload: raw f32 IP search vs SQ8 search with no
rerank (0), the reference rerank (1) and the corrected rerank (2), over the ef sweep.

usage: python tools/sq8_recall.py [--n 1000000] [--nq 1000] [--latent 48] [--sigma 0.15]
"""

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--latent", type=int, default=48)
    ap.add_argument("--sigma", type=float, default=0.15)
    ap.add_argument("--noise", type=float, default=0.01)
    ap.add_argument("--builder", choices=("host", "gpu"), default="host")
    ap.add_argument("--centres", choices=("sphere", "orthant", "subspace"), default="sphere")
    args = ap.parse_args()
    import torch

    import bench as b
    from alayalite_amd import _native
    from workloads.datasets import text_like

    ext = _native._ext
    dev = torch.device("cuda", 0)
    base, q = text_like(args.n, args.nq, args.dim, latent=args.latent, sigma_latent=args.sigma,
                        sigma_noise=args.noise, centres=args.centres)
    bd = torch.from_numpy(base).to(dev)
    qd = torch.from_numpy(q).to(dev)
    gt = b.exact_gt(torch, bd, qd, base, q, metric=1)
    del bd
    t = time.time()
    ix = ext.DeviceIndex(0)
    ix.set_base(base, 1)
    if args.builder == "gpu":
        ix.build_graph(32, 100, 100, 0, 0, 1)
    else:
        ix.set_graph(ext.Graph.build(base, 1, 32, 100, b.host_threads(), 100))
    print(f"n={args.n} centres={args.centres} latent={args.latent} sigma={args.sigma} noise={args.noise}: {args.builder} graph "
          f"{time.time() - t:.1f}s", flush=True)
    mn, mx = ext.sq8_train(base)
    ix.set_sq8(ext.sq8_encode(base, mn, mx, b.host_threads()), mn, mx, ext.host_sq8_order())
    for ef in b.EF_SWEEP:
        raw, _, _ = ix.search(q, 10, ef)
        row = [f"ef={ef:4d}", f"raw {b.recall(raw, gt):.4f}"]
        for mode in (0, 1, 2):
            ids, _, _ = ix.search_sq8(q, 10, ef, mode)
            row.append(f"sq8-rr{mode} {b.recall(ids, gt):.4f}")
        per_q = np.array([len(set(a.tolist()) & set(g.tolist())) for a, g in zip(raw, gt)])
        row.append(f"raw lost(0/10) {np.mean(per_q == 0):.3f} <=5/10 {np.mean(per_q <= 5):.3f}")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
