"""A/B of the visited-table layout (auto / compact 16-bit / wide 32-bit) and size on fixed graphs:
SIFT 1M at ef 85 (10k queries) and GIST 1M at ef 400 (1k queries), device-built graphs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from alayalite_amd import _native
    from workloads.datasets import gist_like, sift_like

    ext = _native._ext
    for name, gen, nq, ef in (("sift", sift_like, 10000, 85), ("gist", gist_like, 1000, 400)):
        base, q = gen(1_000_000, nq)
        dev = ext.DeviceIndex(0)
        dev.set_base(base, 0)
        dev.build_graph(32, 100, 100, 0, 0, 1)
        qd = torch.from_numpy(q).cuda()
        ids = torch.empty((nq, 10), dtype=torch.int32, device="cuda")
        dd = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
        cnt = torch.empty((nq, 4), dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()
        ref = None
        for mode, log2 in ((0, 0), (1, 0), (2, 0), (2, 12), (2, 13), (1, 13), (1, 14)):
            dev.set_visited_mode(mode)
            dev.set_hash_log2(log2)
            for _ in range(3):
                dev.search_device(qd.data_ptr(), nq, 10, ef, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(), st.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(10):
                dev.search_device(qd.data_ptr(), nq, 10, ef, ids.data_ptr(), dd.data_ptr(), cnt.data_ptr(), st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            out = ids.cpu().numpy()
            if ref is None:
                ref = out.copy()
            print(f"{name} ef={ef} mode={mode} log2={log2}: {e0.elapsed_time(e1) / 10:.3f} ms  same_ids={np.array_equal(out, ref)}",
                  flush=True)


if __name__ == "__main__":
    main()
