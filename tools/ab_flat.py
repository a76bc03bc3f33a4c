"""A/B timing of the flat exact k-NN path (config 2 shape: 1M x d U[0,1), 1k queries, k=10) across
builds: mean launch time, QPS and a hash of the ids (equal hashes = same results).
ALAYA_AB_ROOT selects a saved build (e.g. ab/base).  --envs runs environment variants on the same
index, e.g. --envs "ALAYA_FLAT_TILES=0|ALAYA_FLAT_PRESCAN=16|" ('' = the defaults).
usage: python tools/ab_flat.py [--dims 128,64] [--nqs 1000,10000] [--envs ...]"""
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
    ap.add_argument("--dims", default="128")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--nqs", default=None, help="query counts (default --nq)")
    ap.add_argument("--envs", default="", help="'|'-separated variants of comma-separated VAR=VALUE")
    ap.add_argument("--diag", default="", help="ablations to run through flat_diag per variant (e.g. 0,1,3): "
                    "kernel time, fold rounds per block and the single-role scan's per-wave s_memtime split")
    args = ap.parse_args()
    import torch
    from alayalite_amd import _native
    from workloads.datasets import uniform

    ext = _native._ext
    print("engine:", os.path.dirname(_native.__file__), flush=True)
    st = torch.cuda.current_stream()
    variants = [v for v in args.envs.split("|")] if args.envs else [""]
    nqs = [int(x) for x in args.nqs.split(",")] if args.nqs else [args.nq]
    for dim in [int(x) for x in args.dims.split(",")]:
        base, q_all = uniform(args.n, max(nqs), dim, 1, 2)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        for nq in nqs:
            q = np.ascontiguousarray(q_all[:nq])
            qd = torch.from_numpy(q).cuda()
            ids = torch.empty((nq, args.k), dtype=torch.int32, device="cuda")
            dd = torch.empty((nq, args.k), dtype=torch.float32, device="cuda")
            fl = torch.empty((nq,), dtype=torch.int32, device="cuda")

            def run():
                dev.flat_search_device(qd.data_ptr(), nq, args.k, ids.data_ptr(), dd.data_ptr(), fl.data_ptr(),
                                       st.cuda_stream)

            for var in variants:
                saved = {}
                for kv in filter(None, var.split(",")):
                    key, val = kv.split("=", 1)
                    saved[key] = os.environ.get(key)
                    os.environ[key] = val
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.reps):
                    run()
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                h = int(np.bitwise_xor.reduce(ids.cpu().numpy().astype(np.int64).ravel() * 2654435761 % (1 << 31)))
                print(f"flat n {args.n} d {dim} nq {nq} k {args.k} [{var or 'default'}]: {ms:.4f} ms  "
                      f"{nq / ms * 1e3:,.0f} QPS  ids-hash {h}  flagged {int(fl.sum().item())}  "
                      f"contraction {dev.flat_contraction()}", flush=True)
                for ab in [int(x) for x in args.diag.split(",") if x != ""]:
                    mc = torch.zeros((4096 + 2 * 8 * 16384 * 8,), dtype=torch.int32, device="cuda")
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    dev.flat_diag(qd.data_ptr(), nq, args.k, ab, ids.data_ptr(), dd.data_ptr(), fl.data_ptr(),
                                  mc.data_ptr(), st.cuda_stream)
                    b.record(st)
                    torch.cuda.synchronize()
                    m = mc.cpu().numpy()
                    rows = m[4096:].view(np.uint64).reshape(-1, 8).astype(np.float64)
                    rows = rows[rows[:, 0] > 0]
                    msg = ""
                    if len(rows):
                        tot = rows[:, 0].mean()
                        msg = (f"  per-wave ticks {tot:.0f}: wait+barrier {rows[:, 1].mean() / tot:.2f} "
                               f"contraction+test {rows[:, 2].mean() / tot:.2f} candidates {rows[:, 3].mean() / tot:.2f} "
                               f"(max-wave candidates {rows[:, 3].max() / tot:.2f}); records with a candidate "
                               f"{rows[:, 4].mean():.1f} of {rows[:, 6].mean():.1f}, candidates {rows[:, 5].mean():.1f} "
                               f"per wave")
                    nz = m[:4096][m[:4096] > 0]
                    print(f"   diag ablate={ab}: {a.elapsed_time(b):.3f} ms (scan + prescan, no merge)  fold rounds/block "
                          f"{nz.mean() if len(nz) else 0:.1f}{msg}", flush=True)
                for key, val in saved.items():
                    if val is None:
                        os.environ.pop(key, None)
                    else:
                        os.environ[key] = val
        del dev

if __name__ == "__main__":
    main()
