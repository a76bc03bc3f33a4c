"""One-GPU rehearsal of bench.py's N-GPU shard layouts (8-GPU runs are the driver's).

Layout S x G (sharded.Layout): S base-range shards, G = N / S query groups; rank r holds shard r % S
and answers query group r // S (nq / G queries), exchanging inside its group.  S = N is the north
star's pure sharding, S = 1 replicas with the queries split by range.  For each S: build the S shard
graphs on the device exactly as the ranks do (alaya_index_build_graph, deterministic; SQ8: each
shard's own quantizer, the rerank's id-0 entries on the shard holding global row 0), search every
shard on this GPU, merge the per-shard top-k by (dist, global id), pick the smallest ef of the sweep
whose merged recall@10 >= 0.95, then time every (shard, query group) pair a rank would run at that
ef.  Predicted N-GPU QPS = nq / the slowest pair's kernel time (the exchange -- nq/G x k x 8 B per
rank -- is measured by bench.py); efficiency = predicted / (N x the one-GPU QPS of the whole index
on the whole batch at its own ef).

usage: python tools/shard_rehearsal.py [--workload gist|sq8] [--n N] [--nq 10000] [--world 8] [--shards 1,2,4,8]
       (config 4: gist, 1M, 10k queries; config 5: sq8, 10M x 768 IP SQ8 + rerank, 10k queries)
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
    ap.add_argument("--workload", choices=("gist", "sq8"), default="gist")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--nq", type=int, default=10000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch

    import bench as b
    from alayalite_amd import _native
    from alayalite_amd.sharded import merge_reference, shard_range, shard_search
    import workloads.datasets as ds

    ext = _native._ext
    dev = torch.device("cuda", 0)
    sq8 = args.workload == "sq8"
    n = args.n or (10_000_000 if sq8 else 1_000_000)
    metric = 1 if sq8 else 0
    t = time.time()
    base, queries = (ds.text_like(n, args.nq) if sq8 else ds.gist_like(n, args.nq, 960))
    print(f"data {base.shape} in {time.time() - t:.1f}s", flush=True)
    q_all = torch.from_numpy(queries).to(dev)
    t = time.time()
    if sq8:
        base_dev = torch.from_numpy(base).to(dev)
        gt = b.exact_gt(torch, base_dev, q_all, base, queries, metric=1)
        del base_dev
    else:
        gt, _ = b.exact_gt_flat(ext, base, queries, 0)
    torch.cuda.empty_cache()
    print(f"ground truth in {time.time() - t:.1f}s", flush=True)
    nq, K = args.nq, b.K
    stream = torch.cuda.current_stream(dev)
    order = ext.host_sq8_order()

    def build(lo, hi):
        rows = np.ascontiguousarray(base[lo:hi])
        ix = ext.DeviceIndex(0)
        ix.set_base(rows, metric)
        ix.build_graph(b.R, 100, 100, 0, 0, 2)
        if sq8:
            mn, mx = ext.sq8_train(rows)
            ix.set_sq8(ext.sq8_encode(rows, mn, mx, 16), mn, mx, order)
        return ix

    def search(ix, lo, q, ef, timed=False):
        m = q.shape[0]
        ids = torch.empty((m, K), dtype=torch.int32, device=dev)
        dd = torch.empty((m, K), dtype=torch.float32, device=dev)
        cnt = torch.empty((m, 4), dtype=torch.int32, device=dev)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        shard_search(ix, lo, sq8, q, K, ef, ids, dd, cnt, stream.cuda_stream)
        e.record(stream)
        torch.cuda.synchronize()
        if timed:  # the per-(shard, query group) breakdown: time, work and the launch's resident searchers
            c = cnt.cpu().numpy().astype(np.int64)
            g, w = ix.last_launch()
            return a.elapsed_time(e), {"queries": m, "searchers": int(g) * int(w),
                                       "rounds": round(m / max(1, int(g) * int(w)), 3),
                                       "n_dist_sum": int(c[:, 0].sum()), "n_expand_mean": round(float(c[:, 1].mean()), 1),
                                       "n_expand_max": int(c[:, 1].max())}
        return ids.cpu().numpy().astype(np.int64), dd.cpu().numpy().copy(), a.elapsed_time(e)

    results = []
    for S in [int(x) for x in args.shards.split(",")]:
        G = args.world // S
        spans = [shard_range(n, S, s) for s in range(S)]
        t = time.time()
        shards = [(lo, build(lo, hi)) for lo, hi in spans]
        print(f"S={S}: {S} shard graphs in {time.time() - t:.1f}s", flush=True)
        sweep = []

        def probe(ef):
            per = [search(ix, lo, q_all, ef) for lo, ix in shards]
            mi, _ = merge_reference([p[0] for p in per], [p[1] for p in per], [lo for lo, _ in shards], K)
            r = b.recall(mi, gt)
            sweep.append({"ef": ef, "recall": round(r, 4)})
            return r >= 0.95

        ef = b.choose_ef(probe)
        groups = [shard_range(nq, G, g) for g in range(G)]
        for lo, ix in shards:  # warm
            search(ix, lo, q_all[groups[0][0]:groups[0][1]], ef)
        worst = []
        pairs = {}
        for _ in range(args.steps):
            step = []
            for si, (lo, ix) in enumerate(shards):
                for gi, (qa, qb) in enumerate(groups):
                    t_ms, info = search(ix, lo, q_all[qa:qb], ef, timed=True)
                    step.append(t_ms)
                    pairs.setdefault((si, gi), {"shard": si, "group": gi, "ms": [], **info})["ms"].append(t_ms)
            worst.append(max(step))
        ms = float(np.median(worst))
        per_pair = []
        for v in pairs.values():
            v["kernel_ms"] = round(float(np.median(v.pop("ms"))), 3)
            per_pair.append(v)
        row = {"shards": S, "query_groups": G, "ef": ef, "recall": next(x["recall"] for x in sweep if x["ef"] == ef),
               "queries_per_rank": groups[0][1] - groups[0][0], "max_rank_kernel_ms": round(ms, 3),
               "predicted_qps": round(nq / (ms * 1e-3), 1), "per_rank": per_pair, "sweep": sweep}
        if S == 1:  # the one-GPU reference: the whole index, the whole batch
            whole = [search(shards[0][1], 0, q_all, ef, timed=True) for _ in range(args.steps)]
            row["one_gpu_qps"] = round(nq / (float(np.median([w_[0] for w_ in whole])) * 1e-3), 1)
            row["one_gpu"] = {"kernel_ms": round(float(np.median([w_[0] for w_ in whole])), 3), **whole[0][1]}
        results.append(row)
        print(json.dumps(row), flush=True)
        del shards
        torch.cuda.empty_cache()
    one = next((r["one_gpu_qps"] for r in results if "one_gpu_qps" in r), None)
    for r in results:
        if one:
            r["predicted_efficiency"] = round(r["predicted_qps"] / (args.world * one), 3)
    out = {"workload": args.workload, "n": n, "nq": nq, "world": args.world, "one_gpu_qps": one, "layouts": results,
           "note": "kernel-only prediction on one MI355X: every (shard, query group) pair a rank runs, timed in turn; "
                   "the exchange is not included"}
    print(json.dumps(out), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
