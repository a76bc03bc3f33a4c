"""A/B timing of the SQ8 search kernel at small and large batches (768-d IP text-like 1M, device
graph, ef 175) across visited-table sizes: hash_log2 0 = the engine's automatic sizing, else a forced
2^l-slot table (more resident waves per CU, more spills).  Prints the mean launch time and a hash of
the ids (equal hashes = same results).  ALAYA_AB_ROOT selects a saved build (e.g. ab/base).

usage: python tools/ab_sq8.py [--nq 1000,10000] [--hash 0,13,12] [--ef 175] [--n 1000000]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("ALAYA_AB_ROOT"):
    sys.path.insert(0, os.environ["ALAYA_AB_ROOT"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", default="1000,10000")
    ap.add_argument("--hash", default="0,14,13,12")
    ap.add_argument("--ef", type=int, default=175)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch
    from alayalite_amd import _native
    from workloads.datasets import text_like

    ext = _native._ext
    print("engine:", os.path.dirname(_native.__file__), flush=True)
    st = torch.cuda.current_stream()
    nqs = [int(x) for x in args.nq.split(",")]
    base, q = text_like(args.n, max(nqs))
    dev = ext.DeviceIndex(0)
    dev.set_base(base, 1)
    dev.build_graph(32, 100, 100, 0, 0, 2)
    mn, mx = ext.sq8_train(base)
    dev.set_sq8(ext.sq8_encode(base, mn, mx, 16), mn, mx, ext.host_sq8_order())
    for nq in nqs:
        qd = torch.from_numpy(np.ascontiguousarray(q[:nq])).cuda()
        ids = torch.empty((nq, 10), dtype=torch.int32, device="cuda")
        dd = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
        cnt = torch.empty((nq, 4), dtype=torch.int32, device="cuda")
        for hl in [int(x) for x in args.hash.split(",")]:
            dev.set_hash_log2(hl)

            def run():
                dev.search_sq8_device(qd.data_ptr(), 0, nq, 10, args.ef, 1, ids.data_ptr(), dd.data_ptr(),
                                      cnt.data_ptr(), st.cuda_stream)

            for _ in range(2):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            h = int(np.bitwise_xor.reduce(ids.cpu().numpy().astype(np.int64).ravel() * 2654435761 % (1 << 31)))
            c = cnt.cpu().numpy()
            ms = e0.elapsed_time(e1) / args.reps
            print(f"sq8 nq {nq} ef {args.ef} hash_log2 {hl}: {ms:.4f} ms  {nq / ms * 1e3:,.0f} QPS  ids-hash {h}  "
                  f"n_dist {c[:, 0].mean():.1f} n_expand {c[:, 1].mean():.1f}", flush=True)
        dev.set_hash_log2(0)


if __name__ == "__main__":
    main()
