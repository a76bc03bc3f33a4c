"""Per-phase cycle breakdown of the search kernel (diagnostic build with s_memtime stamps).

usage: python tools/profile_phases.py [--n 1000000] [--ef 400] [--nq 1000] [--hash-log2 0]
Prints mean cycles per query for init/descent, pop, adjacency+visited, distances, merge, the
number of expansions after the LDS visited table spilled, and the whole query; and the per-phase
cycles per expansion.  Read the shares, not the absolute time (stamps perturb the schedule).
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
    ap.add_argument("--dim", type=int, default=960)
    ap.add_argument("--ef", type=int, default=400)
    ap.add_argument("--hash-log2", type=int, default=0)
    ap.add_argument("--visited-mode", type=int, default=0, help="0 auto, 1 compact, 2 wide")
    ap.add_argument("--builder", choices=("host", "gpu"), default="host")
    ap.add_argument("--out", default="")
    ap.add_argument("--workload", choices=("gist", "sq8", "sift"), default="gist",
                    help="sq8: config-5 data (768-d IP, device-built graph), stamped SQ8 traversal")
    ap.add_argument("--fine", action="store_true",
                    help="the package was built with -DALAYA_FINE_STAMPS (ALAYA_EXTRA_HIPFLAGS): slots split "
                         "the adjacency wait from the visited phase and the merge's rank/position phase from "
                         "its shift")
    args = ap.parse_args()
    import bench as b  # (puts the tree first on sys.path)

    if os.environ.get("ALAYA_AB_ROOT"):  # a saved (e.g. diagnostic) build of the package instead of the tree's
        sys.path.insert(0, os.environ["ALAYA_AB_ROOT"])
    from alayalite_amd import _native

    print("engine:", os.path.dirname(_native.__file__), flush=True)
    from workloads.datasets import gist_like

    ext = _native._ext
    space = 0
    if args.workload == "sq8":
        from workloads.datasets import text_like

        base, queries = text_like(args.n, args.nq, 768)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 1)
        dev.build_graph(32, 100, 100, 0, 0, 1)
        mn, mx = ext.sq8_train(base)
        dev.set_sq8(ext.sq8_encode(base, mn, mx, b.host_threads()), mn, mx, ext.host_sq8_order())
        space = 1
    elif args.workload == "sift":
        from workloads.datasets import sift_like

        base, queries = sift_like(args.n, args.nq, 128)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        if args.builder == "gpu":
            dev.build_graph(32, 100, 100, 0, 0, 1)
        else:
            g, _ = b.graph_for(ext, base, 100, b.host_threads(), os.path.join(ROOT, "data_cache"), "sift_like_m0")
            dev.set_graph(g)
    else:
        base, queries = gist_like(args.n, args.nq, args.dim)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        if args.builder == "gpu":
            dev.build_graph(32, 100, 100, 0, 0, 2)
        else:
            g, _ = b.graph_for(ext, base, 100, b.host_threads(), os.path.join(ROOT, "data_cache"), "gist")
            dev.set_graph(g)
    if args.hash_log2:
        dev.set_hash_log2(args.hash_log2)
    if args.visited_mode:
        dev.set_visited_mode(args.visited_mode)
    def plain_search():
        if space:
            return dev.search_sq8(queries, 10, args.ef, 0, None)
        return dev.search(queries, 10, args.ef)

    ids0, _, cnt0 = plain_search()
    t = time.time()
    ids0, _, cnt0 = plain_search()
    plain = time.time() - t
    ids, cnt, st = dev.profile_search(queries, 10, args.ef, space)
    assert np.array_equal(ids, ids0)
    names = ["init+descent", "pop", "adj+visited", "distances", "merge", "spilled_expansions", "query_total"]
    if args.fine:
        names = ["init+descent", "pop", "adjacency wait", "distances", "merge shift+tail", "visited+prefetch",
                 "query_total", "merge rank+position"]
    mean = st.mean(0)
    exp = cnt[:, 1].mean()
    print(f"n={args.n} ef={args.ef} nq={args.nq} host-timed plain search {plain*1e3:.2f} ms "
          f"mean n_dist={cnt[:,0].mean():.1f} n_expand={exp:.1f}")
    for i, nme in enumerate(names):
        per = mean[i] / exp if i not in (5, 6) else mean[i]
        print(f"  {nme:20s} mean/query {mean[i]:14.1f}   per expansion {mean[i]/exp:10.1f}")
    if not args.fine:
        print(f"  adjacency prefetch hits {mean[7]:.1f} per query = {mean[7] / exp:.3f} of expansions")
    print(f"  max query_total {st[:,6].max()}  min {st[:,6].min()}  p50 {np.median(st[:,6])}")
    # the launch ends with its slowest query: is the tail more expansions or slower expansions?
    ne = cnt[:, 1].astype(np.float64)
    tot = st[:, 6].astype(np.float64)
    q = [50, 90, 99, 100]
    print("  n_expand percentiles p50/p90/p99/max", [float(np.percentile(ne, x)) for x in q])
    print("  n_dist   percentiles p50/p90/p99/max", [float(np.percentile(cnt[:, 0], x)) for x in q])
    print("  cycles per expansion p50/p90/p99/max", [round(float(np.percentile(tot / ne, x)), 1) for x in q])
    slow = np.argsort(tot)[-5:]
    print("  slowest 5 queries: cycles", tot[slow].astype(np.int64).tolist(), "n_expand", ne[slow].astype(int).tolist(),
          "n_dist", cnt[slow, 0].tolist())
    print(f"  corr(cycles, n_expand) {np.corrcoef(tot, ne)[0, 1]:.3f}")
    if args.out:
        np.save(args.out, st)


if __name__ == "__main__":
    main()
