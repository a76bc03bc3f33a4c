"""How much of a latency-bound batch is the tail?  The persistent search waves take queries from a
work counter in batch order; the launch ends when the last query does, and a latency-bound wave
does not speed up when the others go idle.  On a device-built graph (config 3 sift / config 5 sq8 /
config 4 gist) this times the same queries in several orders (results are order-free: each query's
ids are compared after undoing the permutation):
  batch      -- as given
  shuffled   -- a random permutation (control)
  lpt-exact  -- longest first by the query's own measured n_dist (the bound no predictor can beat)
  lpt-ef<e>  -- longest first by a pre-pass at a small ef (the pre-pass time is reported beside it)
plus the batch tiled 4x (per-query throughput with the tail amortised).

usage: python tools/tail_probe.py [--workload sift] [--nq 10000] [--pre-ef 10,20]
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
    ap.add_argument("--workload", choices=("sq8", "sift", "gist"), default="sift")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--ef", type=int, default=0)
    ap.add_argument("--nq", type=int, default=10000)
    ap.add_argument("--pre-ef", default="10,20")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    from alayalite_amd import _native
    import workloads.datasets as ds

    ext = _native._ext
    gen, n0, ef0, metric, sq8 = {"sq8": (ds.text_like, 10_000_000, 368, 1, True),
                                 "sift": (ds.sift_like, 1_000_000, 70, 0, False),
                                 "gist": (ds.gist_like, 1_000_000, 387, 0, False)}[args.workload]
    n, ef = args.n or n0, args.ef or ef0
    t = time.time()
    base, queries = gen(n, args.nq)
    print(f"data {base.shape} in {time.time() - t:.1f}s", flush=True)
    dev = ext.DeviceIndex(0)
    dev.set_base(base, metric)
    t = time.time()
    dev.build_graph(32, 100, 100, 0, 0, 2)
    print(f"graph in {time.time() - t:.1f}s", flush=True)
    if sq8:
        mn, mx = ext.sq8_train(base)
        dev.set_sq8(ext.sq8_encode(base, mn, mx, 16), mn, mx, ext.host_sq8_order())
    del base
    st = torch.cuda.current_stream()
    nq = args.nq

    def timed(q_np, e, reps):
        m = q_np.shape[0]
        qd = torch.from_numpy(np.ascontiguousarray(q_np)).cuda()
        ids = torch.empty((m, 10), dtype=torch.int32, device="cuda")
        dd = torch.empty((m, 10), dtype=torch.float32, device="cuda")
        cnt = torch.empty((m, 4), dtype=torch.int32, device="cuda")

        def run():
            if sq8:
                dev.search_sq8_device(qd.data_ptr(), 0, m, 10, e, 1, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                      st.cuda_stream)
            else:
                dev.search_device(qd.data_ptr(), m, 10, e, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                  st.cuda_stream)

        for _ in range(2):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps, ids.cpu().numpy(), cnt.cpu().numpy()

    q = np.ascontiguousarray(queries[:nq])
    ms0, ids0, cnt0 = timed(q, ef, args.reps)
    cost = cnt0[:, 0].astype(np.float64)
    print(f"n_dist mean {cost.mean():.1f} p50 {np.percentile(cost, 50):.0f} p99 {np.percentile(cost, 99):.0f} "
          f"max {cost.max():.0f}", flush=True)

    def report(name, perm, extra=""):
        ms, ids, _ = timed(q[perm], ef, args.reps)
        back = np.empty_like(ids)
        back[perm] = ids
        same = np.array_equal(back, ids0)
        print(f"{name:12s} {ms:.3f} ms  {nq / ms * 1e3:,.0f} QPS  ({ms0 / ms:.3f}x batch order)  ids equal {same}{extra}",
              flush=True)
        return ms

    print(f"{'batch':12s} {ms0:.3f} ms  {nq / ms0 * 1e3:,.0f} QPS", flush=True)
    report("shuffled", np.random.default_rng(0).permutation(nq))
    report("lpt-exact", np.argsort(-cost, kind="stable"))
    for pe in [int(x) for x in args.pre_ef.split(",") if x]:
        ms_pre, _, cnt_pre = timed(q, pe, args.reps)
        pc = cnt_pre[:, 0].astype(np.float64)
        rho = np.corrcoef(np.argsort(np.argsort(pc)), np.argsort(np.argsort(cost)))[0, 1]
        report(f"lpt-ef{pe}", np.argsort(-pc, kind="stable"),
               f"  (pre-pass {ms_pre:.3f} ms, rank corr {rho:.2f})")
    ms4, _, _ = timed(np.tile(q, (4, 1)), ef, max(2, args.reps // 4))
    print(f"{'tiled x4':12s} {ms4:.3f} ms  {4 * nq / ms4 * 1e3:,.0f} QPS  (per query {ms4 / 4:.3f} ms-equivalent per "
          f"{nq}: {ms0 / (ms4 / 4):.3f}x)", flush=True)


if __name__ == "__main__":
    main()
