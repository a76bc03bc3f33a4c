"""Committed golden vectors (tests/golden/, made by tools/make_golden.py): the CPU restatement
must reproduce them on CPU, and the device path must reproduce them bit for bit on the MI355X."""

import glob
import hashlib
import os

import numpy as np
import pytest

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def _base(name):
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "make_golden", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return {"c1_l2": mg.c1_data, "ip_96": mg.ip_data, "cos_100": mg.cos_data}[name]()


def _load(path):
    z = np.load(path, allow_pickle=False)
    name = os.path.basename(path)[:-4]
    base, queries = _base(name)
    assert hashlib.md5(base.tobytes()).hexdigest() == str(z["base_md5"])
    assert np.array_equal(queries, z["queries"])
    return z, base


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(orc, path):
    z, base = _load(path)
    view = orc.IndexView(base, z["l0"], z["levels"], z["upper_off"], z["upper_edges"],
                         int(z["upper_R"]), int(z["ep"]), metric=int(z["metric"]))
    for ef in z["efs"]:
        for i, q in enumerate(z["queries"]):
            ids, d, cnt = view.search(q, 10, int(ef), with_counters=True)
            assert np.array_equal(ids, z[f"ids_ef{ef}"][i])
            assert np.array_equal(d.view(np.uint32), z[f"dists_ef{ef}"][i].view(np.uint32))
            assert tuple(cnt) == tuple(z[f"counters_ef{ef}"][i])


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_builder_reproduces_golden_graph(native, path):
    z, base = _load(path)
    g = native.Graph.build(base, int(z["metric"]), 32, 100, 1, 100)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    assert np.array_equal(l0, z["l0"]) and np.array_equal(levels, z["levels"])
    assert np.array_equal(ue, z["upper_edges"]) and ep == int(z["ep"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_device_reproduces_golden(native, path):
    z, base = _load(path)
    dev = native.DeviceIndex(0)
    dev.set_base(base, int(z["metric"]))
    dev.set_graph(native.Graph.from_arrays(z["l0"], z["levels"], z["upper_off"], z["upper_edges"],
                                           int(z["upper_R"]), int(z["ep"])))
    for ef in z["efs"]:
        ids, d, cnt = dev.search(z["queries"], 10, int(ef))
        assert np.array_equal(ids, z[f"ids_ef{ef}"]), ef
        assert np.array_equal(d.view(np.uint32), z[f"dists_ef{ef}"].view(np.uint32)), ef
        assert np.array_equal(cnt.astype(np.uint64), z[f"counters_ef{ef}"]), ef
