"""Diagnostics for the flat MFMA scan: full kernel vs MFMA-only ablation, merges per block."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("ALAYA_AB_ROOT"):  # a saved build (e.g. ab/base)
    sys.path.insert(0, os.environ["ALAYA_AB_ROOT"])
import torch
from alayalite_amd import _native
from workloads.datasets import uniform

base, q = uniform(1_000_000, 1000, 128, 1, 2)
dev = _native._ext.DeviceIndex(0)
dev.set_base(base, 0)
d = torch.device("cuda", 0)
qd = torch.from_numpy(q).to(d)
ids = torch.zeros((1000, 10), dtype=torch.int32, device=d)
ds = torch.zeros((1000, 10), dtype=torch.float32, device=d)
fl = torch.zeros((1000,), dtype=torch.int32, device=d)
mc = torch.zeros((4096 + 2 * 4 * 4096 * 4,), dtype=torch.int32, device=d)
stream = torch.cuda.current_stream(d).cuda_stream
for ablate in (0, 1, 2, 0, 1, 2):
    mc.zero_()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    dev.flat_diag(qd.data_ptr(), 1000, 10, ablate, ids.data_ptr(), ds.data_ptr(), fl.data_ptr(), mc.data_ptr(), stream)
    b.record()
    torch.cuda.synchronize()
    m = mc.cpu().numpy()
    kc = 1 if os.environ.get("ALAYA_FLAT_WS2") == "0" else 2  # consumer waves per producer
    sm = mc[4096:].cpu().numpy().view(np.uint64).reshape(-1, 4)[:1024 * kc].astype(np.float64)
    st = sm; tot = st[:, 0].mean()
    print(f"   per-wave memtime ticks: total {tot:.0f} append {st[:,1].mean()/tot:.2f} fold {st[:,2].mean()/tot:.2f} (max-wave {st[:,2].max()/tot:.2f}) barrier/wait {st[:,3].mean()/tot:.2f}")
    pr = mc[4096:].cpu().numpy().view(np.uint64).reshape(-1, 4)[1024 * kc:1024 * kc + 1024].astype(np.float64)
    if ablate == 0 and pr[:, 0].mean() > 0:  # warp-specialised scan: producer rows
        pt = pr[:, 0].mean()
        print(f"   producers: total {pt:.0f} wait-for-slot {pr[:,1].mean()/pt:.2f} wait-for-staging {pr[:,2].mean()/pt:.2f}")
    print(f"ablate={ablate} scan {a.elapsed_time(b):.3f} ms  merges/block mean {m[:256].mean():.1f} max {m[:256].max()}")
