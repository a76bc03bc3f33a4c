"""Driver for the pybind module under AddressSanitizer (tools/run_sanitizers.sh): exercises the
module's host code -- numpy buffer ownership, dtype casts, the host mirrors -- through the public
API.  With a GPU: Client/Index fit, batch_search(_with_distance), search, insert, remove,
get_data_by_id, save / load for float32 / int8 / float64 rows, L2 / IP / COS, an SQ8 index, and
the error paths; without one (this container): the Graph class (host build, save, load, arrays,
from_arrays), sq8_train / sq8_encode and the "no device" error path.
usage: <asan python> pybind_driver.py <package root> <tmp dir>"""
import os
import sys

sys.path.insert(0, sys.argv[1])
os.environ["ALAYA_SKIP_TORCH_INIT"] = "1"  # the driver never uses torch: keep it out of the process
import numpy as np  # noqa: E402

from alayalite_amd import _native  # noqa: E402

ext = _native._ext
tmp = sys.argv[2]
rng = np.random.default_rng(0)
print("engine:", _native.__file__, flush=True)

# ---- host-only surface ------------------------------------------------------------------------
base = rng.random((3000, 40), dtype=np.float32)
for threads in (1, 4):
    g = ext.Graph.build(base, 0, 32, 60, threads, 100)
    l0, levels, off, ue, ep, ur, eps = g.arrays()
    path = os.path.join(tmp, f"g{threads}.index")
    g.save(path, 4, 4000)
    g2 = ext.Graph.load(path, 4)
    assert np.array_equal(g2.arrays()[0], l0)
    g3 = ext.Graph.from_arrays(l0, levels, off, ue, ur, ep)
    assert np.array_equal(g3.arrays()[3], ue)
    g4 = ext.Graph.from_arrays(l0, None, None, None, 0, 0, np.array([0, 5], np.uint32))
    assert g4.arrays()[6].tolist() == [0, 5]
mn, mx = ext.sq8_train(base)
codes = ext.sq8_encode(base, mn, mx, 4)
assert codes.shape == base.shape and codes.dtype == np.uint8
for bad in (lambda: ext.Graph.load(os.path.join(tmp, "missing.index"), 4),
            lambda: ext.Graph.from_arrays(l0[:, :3] * 0 + 99999, None, None, None, 0, 0, np.zeros(1, np.uint32))):
    try:
        bad()
    except (RuntimeError, ValueError):
        pass
print("host surface ok", flush=True)

if ext.device_count() == 0:
    try:
        ext.DeviceIndex(0)
        raise SystemExit("expected the no-device error")
    except RuntimeError:
        pass
    print("no device: index paths skipped", flush=True)
    sys.exit(0)

# ---- the Index API (GPU) ----------------------------------------------------------------------
import alayalite_amd  # noqa: E402

client = alayalite_amd.Client(os.path.join(tmp, "db"))
for dtype, metric, quant in ((np.float32, "l2", "none"), (np.float32, "ip", "none"), (np.float32, "cosine", "none"),
                             (np.int8, "l2", "none"), (np.float64, "ip", "none"), (np.float32, "ip", "sq8")):
    name = f"i_{np.dtype(dtype).name}_{metric}_{quant}"
    rows = (rng.integers(-60, 60, (2000, 32)) if dtype == np.int8 else rng.standard_normal((2000, 32))).astype(dtype)
    qs = rows[:17].copy() + (0 if dtype == np.int8 else dtype(0.01))
    idx = client.create_index(name, capacity=2100, data_type=dtype, metric=metric, quantization_type=quant)
    idx.fit(rows.copy(), ef_construction=60, num_threads=2)
    ids = idx.batch_search(qs.copy(), 10, 50)
    ids2, d2 = idx.batch_search_with_distance(qs.copy(), 10, 50)
    one = idx.search(qs[0].copy(), 10, 50)
    assert ids.shape == (17, 10) and one.shape == (10,)
    if quant == "none":
        new = idx.insert(rows[5].copy(), 40)
        idx.remove(3)
        _ = idx.get_data_by_id(int(new))
        idx.batch_search(qs.copy(), 5, 30)
    client.save_index(name)
    again = alayalite_amd.Client(os.path.join(tmp, "db")).get_index(name)
    again.batch_search(qs.copy(), 10, 50)
    for bad in (lambda: idx.batch_search(qs[:, :5].copy(), 10, 50), lambda: idx.search(qs[0][:3].copy(), 10, 50)):
        try:
            bad()
        except (RuntimeError, ValueError):
            pass
    print(name, "ok", flush=True)
print("index API ok", flush=True)
