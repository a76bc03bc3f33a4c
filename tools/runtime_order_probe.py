"""Which first use of the GPU works when torch (bundled HIP runtime) and the engine share a process?

Each case runs in a fresh child process (nothing initialised when it starts):
  torch-first   import torch, torch.cuda.is_available(), then the engine
  engine-first  import torch (libraries loaded, nothing initialised), the engine's first device call,
                then torch's
  no-torch      the engine alone (ALAYA_SKIP_TORCH_INIT=1, torch never imported)
and reports whether the engine saw a device, whether torch did, and whether an engine search on
torch-allocated device memory returned the same ids as the engine's host-buffer search.

usage: python tools/runtime_order_probe.py
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path.insert(0, ROOT)
case = sys.argv[1]
out = {"case": case}
import numpy as np
if case != "no-torch":
    import torch
    if case == "torch-first":
        out["torch_available"] = torch.cuda.is_available()
from alayalite_amd import _native
ext = _native._ext
out["engine_devices"] = ext.device_count()
rng = np.random.default_rng(0)
base = rng.random((2000, 32), dtype=np.float32)
q = rng.random((8, 32), dtype=np.float32)
dev = ext.DeviceIndex(0)
dev.set_base(base, 0)
dev.build_graph(32, 100, 100, 0, 0, 2)
ids, _, _ = dev.search(q, 10, 40)
out["engine_search"] = True
if case != "no-torch":
    if case == "engine-first":
        out["torch_available"] = torch.cuda.is_available()
    qd = torch.from_numpy(q).cuda()
    i2 = torch.empty((8, 10), dtype=torch.int32, device="cuda")
    d2 = torch.empty((8, 10), dtype=torch.float32, device="cuda")
    c2 = torch.empty((8, 4), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    dev.search_device(qd.data_ptr(), 8, 10, 40, i2.data_ptr(), d2.data_ptr(), c2.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    out["device_buffers_equal"] = bool(np.array_equal(i2.cpu().numpy().astype(np.uint32), ids))
print("RESULT " + json.dumps(out), flush=True)
"""


def main():
    results = []
    for case in ("torch-first", "engine-first", "no-torch"):
        env = dict(os.environ)
        env["ALAYA_SKIP_TORCH_INIT"] = "1"  # the child chooses the order itself
        p = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT)), case], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        r = json.loads(line[0][7:]) if line else {"case": case, "error": (p.stderr or p.stdout)[-600:]}
        r["rc"] = p.returncode
        print(json.dumps(r), flush=True)
        results.append(r)


if __name__ == "__main__":
    main()
