"""A/B timing of the flat exact k-NN path (config 2 shape: 1M x d U[0,1), 1k queries, k=10) across
builds: mean launch time, QPS and a hash of the ids (equal hashes = same results).
ALAYA_AB_ROOT selects a saved build (e.g. ab/base).  usage: python tools/ab_flat.py [--dims 128,64]"""
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
    args = ap.parse_args()
    import torch
    from alayalite_amd import _native
    from workloads.datasets import uniform

    ext = _native._ext
    print("engine:", os.path.dirname(_native.__file__), flush=True)
    st = torch.cuda.current_stream()
    for dim in [int(x) for x in args.dims.split(",")]:
        base, q = uniform(args.n, args.nq, dim, 1, 2)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        qd = torch.from_numpy(q).cuda()
        ids = torch.empty((args.nq, args.k), dtype=torch.int32, device="cuda")
        dd = torch.empty((args.nq, args.k), dtype=torch.float32, device="cuda")
        fl = torch.empty((args.nq,), dtype=torch.int32, device="cuda")

        def run():
            dev.flat_search_device(qd.data_ptr(), args.nq, args.k, ids.data_ptr(), dd.data_ptr(), fl.data_ptr(),
                                   st.cuda_stream)

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
        print(f"flat n {args.n} d {dim} nq {args.nq} k {args.k}: {ms:.4f} ms  {args.nq / ms * 1e3:,.0f} QPS  "
              f"ids-hash {h}  flagged {int(fl.sum().item())}", flush=True)
        del dev


if __name__ == "__main__":
    main()
