"""Launch-shape sweep of the graph search on a device-built graph: config 5 (sq8: 10M x 768 IP rows,
workloads.datasets.text_like seeds 7/8, SQ8 search + reference rerank), config 3 (sift: 1M x 128 L2)
or config 4 (gist: 1M x 960 L2), at a fixed ef over 10k (and 1k) queries, for each combination of
searchers per workgroup (ALAYA_SEARCH_WAVES), cap on resident searchers per CU
(ALAYA_MAX_WAVES_PER_CU) and visited table (a negative value = a fixed log2 via set_hash_log2).  Prints the mean launch time, QPS, mean
n_dist and a hash of the ids (equal hashes = identical results).

usage: python tools/shape_sweep.py [--workload sq8] [--n 10000000] [--ef 340] [--waves 1,2,4] [--max-waves 0,12,16] [--table 0,-12]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("ALAYA_AB_ROOT"):  # A/B: a saved build of the package (e.g. ab/base) instead of the tree's
    sys.path.insert(0, os.environ["ALAYA_AB_ROOT"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("sq8", "sift", "gist"), default="sq8")
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--ef", type=int, default=0)
    ap.add_argument("--nq", default="10000,1000")
    ap.add_argument("--waves", default="0", help="searchers per workgroup; 0 = the engine's choice")
    ap.add_argument("--visited", default="0", help="visited-table layouts: 0 auto, 1 compact, 2 wide")
    ap.add_argument("--max-waves", default="0", help="caps on resident searchers per CU (ALAYA_MAX_WAVES_PER_CU); 0 = none")
    ap.add_argument("--table", default="0", help="slots per ef targets (0 = default policy); negative = fixed log2")
    ap.add_argument("--spill-table", default="d",
                    help="ALAYA_SPILL_TABLE values: d = the engine's default, 0 = bitset second level, 6..16 = log2 entries")
    ap.add_argument("--env-sweep", default="", help="NAME=v1,v2,...: also sweep an environment knob ('-' = unset)")
    ap.add_argument("--envs", default="", help="environment variants: comma-separated, each '-' (none) or "
                                               "NAME=VAL+NAME=VAL...; applied on top of --env-sweep")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--order", default="batch",
                    help="query orders (comma-separated): batch; xcd = queries grouped by their nearest of 256 "
                         "pivot rows, group chunk x at positions = x mod 8 (the first round's XCD); sorted = "
                         "grouped contiguously.  ids are compared in batch order")
    args = ap.parse_args()
    import torch

    from alayalite_amd import _native
    import workloads.datasets as ds

    ext = _native._ext
    print("engine:", os.path.dirname(_native.__file__), flush=True)
    gen, n0, ef0, metric, sq8 = {"sq8": (ds.text_like, 10_000_000, 340, 1, True),
                                 "sift": (ds.sift_like, 1_000_000, 70, 0, False),
                                 "gist": (ds.gist_like, 1_000_000, 387, 0, False)}[args.workload]
    n, ef = args.n or n0, args.ef or ef0
    t = time.time()
    base, queries = gen(n, 10000)
    print(f"data {base.shape} in {time.time() - t:.1f}s", flush=True)
    dev = ext.DeviceIndex(0)
    dev.set_base(base, metric)
    t = time.time()
    dev.build_graph(32, 100, 100, 0, 0, 2)
    print(f"graph in {time.time() - t:.1f}s", flush=True)
    if sq8:
        mn, mx = ext.sq8_train(base)
        dev.set_sq8(ext.sq8_encode(base, mn, mx, 16), mn, mx, ext.host_sq8_order())
    piv = base[np.random.default_rng(11).choice(base.shape[0], 256, replace=False)].astype(np.float32)
    del base

    def order_perm(kind, nq):
        if kind == "batch":
            return np.arange(nq)
        q = queries[:nq].astype(np.float32)
        sc = q @ piv.T if metric == 1 else 2 * (q @ piv.T) - (piv * piv).sum(1)[None, :]
        key = np.argmax(sc, axis=1)
        srt = np.argsort(key, kind="stable")
        if kind == "sorted":
            return srt
        chunks = np.array_split(srt, 8)  # chunk x -> positions x, x + 8, ...
        perm = np.empty(nq, np.int64)
        for x, c in enumerate(chunks):
            pos = np.arange(x, nq, 8)[: len(c)]
            perm[pos] = c[: len(pos)]
        return perm

    st = torch.cuda.current_stream()
    for nq, order in [(int(x), o) for x in args.nq.split(",") for o in args.order.split(",")]:
        perm = order_perm(order, nq)
        qd = torch.from_numpy(np.ascontiguousarray(queries[:nq][perm])).cuda()
        ids = torch.empty((nq, 10), dtype=torch.int32, device="cuda")
        dd = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
        cnt = torch.empty((nq, 4), dtype=torch.int32, device="cuda")
        env_name, env_vals = (args.env_sweep.split("=", 1)[0], args.env_sweep.split("=", 1)[1].split(",")) \
            if args.env_sweep else ("", ["-"])
        variants = args.envs.split(",") if args.envs else ["-"]
        known = {kv.split("=", 1)[0] for v_ in variants if v_ != "-" for kv in v_.split("+")}
        for w, mw, vm, stb, ev, var in [(w, mw, vm, stb, ev, var) for w in args.waves.split(",")
                                        for mw in args.max_waves.split(",") for vm in args.visited.split(",")
                                        for stb in args.spill_table.split(",") for ev in env_vals for var in variants]:
            if env_name:
                os.environ.pop(env_name, None)
                if ev != "-":
                    os.environ[env_name] = ev
            for k in known:
                os.environ.pop(k, None)
            if var != "-":
                for kv in var.split("+"):
                    k, v_ = kv.split("=", 1)
                    os.environ[k] = v_
            os.environ.pop("ALAYA_SPILL_TABLE", None)
            if stb != "d":
                os.environ["ALAYA_SPILL_TABLE"] = stb
            dev.set_visited_mode(int(vm))
            os.environ.pop("ALAYA_SEARCH_WAVES", None)
            if w != "0":
                os.environ["ALAYA_SEARCH_WAVES"] = w
            os.environ.pop("ALAYA_MAX_WAVES_PER_CU", None)
            if mw != "0":
                os.environ["ALAYA_MAX_WAVES_PER_CU"] = mw
            for tb in [int(x) for x in args.table.split(",")]:
                os.environ.pop("ALAYA_VISITED_TABLE_EF", None)
                dev.set_hash_log2(0)
                if tb > 0:
                    os.environ["ALAYA_VISITED_TABLE_EF"] = str(tb)
                elif tb < 0:
                    dev.set_hash_log2(-tb)

                def run():
                    if sq8:
                        dev.search_sq8_device(qd.data_ptr(), 0, nq, 10, ef, 1, ids.data_ptr(), dd.data_ptr(),
                                              cnt.data_ptr(), st.cuda_stream)
                    else:
                        dev.search_device(qd.data_ptr(), nq, 10, ef, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                          st.cuda_stream)

                for _ in range(2):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.reps):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                ids_b = np.empty((nq, 10), np.int64)
                ids_b[perm] = ids.cpu().numpy()
                h = int(np.bitwise_xor.reduce(ids_b.ravel() * 2654435761 % (1 << 31)))
                c = cnt.cpu().numpy()
                hs = ""
                if hasattr(dev, "help_stats"):
                    st_ = dev.help_stats()
                    m, x, hr = (tuple(st_) + (0, 0))[:3]
                    if m:
                        hs = (f"  memo {m / max(1, int(c[:, 0].sum())):.3f} of distances, "
                              f"{x / max(1, int(c[:, 1].sum())):.3f} of expansions, "
                              f"helper rows / memo hits {hr / max(1, m):.2f}")
                print(f"nq {nq}{'' if order == 'batch' else ' order ' + order} waves {w} max/CU {mw} visited {vm} table {tb} spill-table {stb}"
                      f"{f' {env_name}={ev}' if env_name else ''}{f' [{var}]' if var != '-' else ''}: {ms:.3f} ms  {nq / ms * 1e3:,.0f} QPS  ids-hash {h}  "
                      f"n_dist {c[:, 0].mean():.1f} n_expand {c[:, 1].mean():.1f}{hs}", flush=True)
    os.environ.pop("ALAYA_SEARCH_WAVES", None)
    os.environ.pop("ALAYA_MAX_WAVES_PER_CU", None)
    os.environ.pop("ALAYA_SPILL_TABLE", None)


if __name__ == "__main__":
    main()
