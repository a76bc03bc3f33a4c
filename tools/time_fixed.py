"""Kernel time on fixed, deterministic (device-built) graphs, for A/B across builds and search
modes: SIFT 1M ef 85 (10k and 1k queries), GIST 1M ef 400 (1k), 768-d IP SQ8 1M ef 175 (1k).

usage: python tools/time_fixed.py [--visited 0,2] [--only sift,gist,sq8,sift1k]
Prints per workload and visited-table mode (0 auto, 1 compact, 2 wide) the mean launch time and a
hash of the returned ids (equal hashes across modes = same results)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("ALAYA_AB_ROOT"):  # A/B: a saved build of the package (e.g. ab/base) instead of the tree's
    sys.path.insert(0, os.environ["ALAYA_AB_ROOT"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--visited", default="0")
    ap.add_argument("--only", default="sift,sift1k,gist,sq8")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from alayalite_amd import _native
    from workloads.datasets import gist_like, sift_like, text_like

    ext = _native._ext
    print("engine:", os.path.dirname(_native.__file__), flush=True)
    st = torch.cuda.current_stream()
    modes = [int(m) for m in args.visited.split(",")]
    only = set(args.only.split(","))
    cache = {}
    for name, gen, nq, ef, metric, sq8 in (("sift", sift_like, 10000, 85, 0, False),
                                           ("sift1k", sift_like, 1000, 85, 0, False),
                                           ("gist", gist_like, 1000, 400, 0, False),
                                           ("sq8", text_like, 1000, 175, 1, True)):
        if name not in only:
            continue
        key = gen.__name__
        if key not in cache:
            base, q = gen(1_000_000, 10000)
            dev = ext.DeviceIndex(0)
            dev.set_base(base, metric)
            dev.build_graph(32, 100, 100, 0, 0, 2)
            if sq8:
                mn, mx = ext.sq8_train(base)
                dev.set_sq8(ext.sq8_encode(base, mn, mx, 16), mn, mx, ext.host_sq8_order())
            cache[key] = (dev, q)
        dev, q = cache[key]
        q = q[:nq]
        qd = torch.from_numpy(np.ascontiguousarray(q)).cuda()
        ids = torch.empty((nq, 10), dtype=torch.int32, device="cuda")
        dd = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
        cnt = torch.empty((nq, 4), dtype=torch.int32, device="cuda")

        def run():
            if sq8:
                dev.search_sq8_device(qd.data_ptr(), 0, nq, 10, ef, 1, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(),
                                      st.cuda_stream)
            else:
                dev.search_device(qd.data_ptr(), nq, 10, ef, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(), st.cuda_stream)

        for mode in modes:
            dev.set_visited_mode(mode)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            h = int(np.bitwise_xor.reduce(ids.cpu().numpy().astype(np.int64).ravel() * 2654435761 % (1 << 31)))
            c = cnt.cpu().numpy()
            print(f"{name} visited {mode}: {e0.elapsed_time(e1) / args.reps:.4f} ms  ids-hash {h}  "
                  f"n_dist {c[:, 0].mean():.1f} n_expand {c[:, 1].mean():.1f}", flush=True)
        dev.set_visited_mode(0)


if __name__ == "__main__":
    main()
