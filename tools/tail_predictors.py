"""Which observable predicts a query's remaining search work?  A plain-Python best-first search
(pool of ef, visited set; not the bit-exact LinearPool) on a host-built SIFT-like graph records, at
expansion X, the pool's unchecked entries, the first unchecked position, insertions over the last
five expansions, the best / worst pool distance and the pool size, and ranks each against the
expansions still to come (Spearman).  DESIGN.md §8 "Next" (the batch tail).

usage: python tools/tail_predictors.py [--n 300000] [--nq 2000] [--ef 70]
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
    ap.add_argument("--n", type=int, default=300_000)
    ap.add_argument("--nq", type=int, default=2000)
    ap.add_argument("--ef", type=int, default=70)
    args = ap.parse_args()
    import workloads.datasets as ds
    from alayalite_amd import _native

    base, q = ds.sift_like(args.n, args.nq)
    g = _native._ext.Graph.build(base, 0, 32, 100, 8, 100)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    R = 32
    l0 = np.asarray(l0).reshape(-1, R)
    levels, off, ue = np.asarray(levels), np.asarray(off), np.asarray(ue)

    def d2(qv, ids):
        x = base[ids] - qv
        return (x * x).sum(1)

    marks = (10, 20, 30, 40)

    def search(qv, ef):
        u = int(ep)
        cur = float(d2(qv, [u])[0])
        for lev in range(int(levels[u]), 0, -1):
            changed = True
            while changed:
                changed = False
                lst = ue[off[u] + (lev - 1) * upper_r: off[u] + lev * upper_r]
                lst = lst[lst != 0xFFFFFFFF]
                if len(lst) == 0:
                    break
                dd = d2(qv, lst)
                i = int(np.argmin(dd))
                if dd[i] < cur:
                    cur, u, changed = float(dd[i]), int(lst[i]), True
        pool = [(cur, u, False)]
        vis = {u}
        nexp, feats, recent = 0, {}, []
        while True:
            idx = next((i for i, p in enumerate(pool) if not p[2]), None)
            if idx is None:
                break
            d, u, _ = pool[idx]
            pool[idx] = (d, u, True)
            nexp += 1
            nb = l0[u]
            fresh = [v for v in nb[nb != 0xFFFFFFFF] if v not in vis]
            vis.update(fresh)
            ins = 0
            if fresh:
                for v, dv in zip(fresh, d2(qv, np.array(fresh))):
                    if len(pool) < ef or dv < pool[-1][0]:
                        pool.append((float(dv), int(v), False))
                        pool.sort(key=lambda t: t[0])
                        pool = pool[:ef]
                        ins += 1
            recent.append(ins)
            if nexp in marks:
                unchecked = sum(1 for p in pool if not p[2])
                first = next((i for i, p in enumerate(pool) if not p[2]), ef)
                feats[nexp] = (unchecked, first, sum(recent[-5:]), pool[0][0], pool[-1][0], len(pool))
        return nexp, feats

    t = time.time()
    res = [search(q[i], args.ef) for i in range(args.nq)]
    print(f"{args.nq} searches in {time.time() - t:.1f}s", flush=True)
    tot = np.array([r[0] for r in res], float)

    def rank_corr(a, b):
        return float(np.corrcoef(np.argsort(np.argsort(a)), np.argsort(np.argsort(b)))[0, 1])

    names = ["unchecked", "first_unchecked", "inserted_last5", "best", "worst", "pool_size"]
    for x in marks:
        ok = [i for i, r in enumerate(res) if x in r[1]]
        rem = tot[ok] - x
        f = np.array([res[i][1][x] for i in ok], float)
        print(f"X={x} ({len(ok)} queries): " + "  ".join(f"{n} {rank_corr(f[:, k], rem):+.2f}" for k, n in enumerate(names)))
    print(f"expansions mean {tot.mean():.1f}, p50/p90/p99 {np.percentile(tot, [50, 90, 99])}")


if __name__ == "__main__":
    main()
