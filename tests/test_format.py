"""On-disk format parity, checked with the test-side codec in
tests/refformat.py (written from graph.hpp:165-238, overlay_graph.hpp:151-194,
sequential_storage.hpp:110-142, raw_space.hpp:219-250, sq8_space.hpp:213-251, sq8.hpp:161-177,
schema.py:103-112):

  * engine-written files decode field by field (graph with u32 and u64 ids, with and without the
    overlay; raw.data; SQ8 data; schema.json; the storage bitmaps after remove());
  * files hand-assembled in the reference's layout load into the engine and search identically to
    the oracle's search of the same arrays -- including the reference's width quirks (max_nbrs_
    written with sizeof(IDType) bytes, 64-bit overlay lists truncated to their first half).
"""

import json
import os

import numpy as np
import pytest

import refformat as rf

NONE = 0xFFFFFFFF


def _ids_as(a, dtype):
    """Engine ids (uint32, NONE = -1) in an IDType array: -1 becomes that type's all-ones value."""
    a = np.asarray(a)
    return np.where(a == NONE, np.iinfo(dtype).max, a.astype(np.uint64)).astype(dtype)


def _oracle_graph(orc, base, metric=0):
    return orc.build_hnsw(base, metric, 32, 100, 100)  # l0, levels, off, ue, ep, R


# ---- graph files (host only) ----------------------------------------------------------------------
@pytest.mark.parametrize("id_bytes", [4, 8])
def test_engine_graph_file_decodes(native, orc, c1, tmp_path, id_bytes):
    base, _ = c1
    l0, levels, off, ue, ep, R = _oracle_graph(orc, base)
    g = native.Graph.from_arrays(l0, levels, off, ue, R, ep)
    path = str(tmp_path / "g.index")
    g.save(path, id_bytes, 1500)
    d = rf.read_graph(path, id_bytes)
    assert len(d["eps"]) == 0 and d["max_nodes"] == 1500 and d["max_nbrs"] == 32
    assert (d["item_size"], d["aligned_item_size"]) == (32 * id_bytes, 32 * id_bytes)
    assert (d["capacity"], d["pos"], d["alignment"]) == (1500, 1000, 64)
    idt = np.uint32 if id_bytes == 4 else np.uint64
    full = np.iinfo(idt).max
    want = _ids_as(l0, idt)
    assert np.array_equal(d["rows"][:1000], want)
    assert (d["rows"][1000:] == full).all()  # Graph's storage is initialised with -1 (graph.hpp:65-68)
    assert d["valid"][:1000].all() and not d["valid"][1000:].any()
    ov = d["overlay"]
    assert (ov["node_num"], ov["max_nbrs"], ov["ep"]) == (1500, 32, ep)
    lists = rf.overlay_lists(levels, off, ue, R)
    for i in range(1500):
        lst = ov["lists"][i]
        if i >= 1000 or levels[i] == 0:
            assert len(lst) == 0
            continue
        assert len(lst) == levels[i] * 32
        want = _ids_as(lists[i], idt)
        if id_bytes == 4:
            assert np.array_equal(lst, want)
        else:  # cur * 4 bytes of a 64-bit list: the first half of the entries, the rest stays -1
            h = len(lst) // 2
            assert np.array_equal(lst[:h], want[:h]) and (lst[h:] == full).all()


@pytest.mark.parametrize("id_bytes", [4, 8])
def test_reference_layout_graph_loads(native, orc, tmp_path, id_bytes):
    """A graph file assembled by the codec in the reference's layout loads into the engine with the
    arrays the reference's own Graph::load would hold (u64: overlay lists cut to their first half,
    the upper bytes of the 64-bit max_nbrs_ field ignored)."""
    rng = np.random.default_rng(3)
    base = rng.random((700, 40), dtype=np.float32)
    l0, levels, off, ue, ep, R = _oracle_graph(orc, base)
    lists = rf.overlay_lists(levels, off, ue, R)
    wide = lambda a: _ids_as(a, np.uint64)  # noqa: E731
    path = str(tmp_path / "ref.index")
    rf.write_graph(path, id_bytes, l0 if id_bytes == 4 else wide(l0), 900,
                   overlay=(ep, lists if id_bytes == 4 else [wide(x) for x in lists]), max_nbrs_pad=0xDEADBEEF)
    g = native.Graph.load(path, id_bytes)
    gl0, glev, goff, gue, gep, gR, _ = g.arrays()
    assert np.array_equal(gl0, l0) and np.array_equal(glev, levels) and gep == ep and gR == R
    for i in np.nonzero(levels)[0]:
        got = gue[goff[i]: goff[i] + levels[i] * R]
        want = lists[i].copy()
        if id_bytes == 8:
            want[len(want) // 2:] = NONE
        assert np.array_equal(got, want), i


def test_nsg_style_graph_file(native, tmp_path):
    """A graph without an overlay (NSG-style entry points, graph.hpp:153-156): nep > 0, no bytes
    after the storage."""
    l0 = np.full((50, 32), NONE, np.uint32)
    l0[:, 0] = (np.arange(50) + 1) % 50
    path = str(tmp_path / "nsg.index")
    rf.write_graph(path, 4, l0, 64, eps=[3, 9, 3])
    g = native.Graph.load(path, 4)
    a = g.arrays()
    assert np.array_equal(a[0], l0) and a[1] is None and list(a[-1]) == [3, 9, 3]
    g.save(str(tmp_path / "again.index"), 4, 64)
    d = rf.read_graph(str(tmp_path / "again.index"), 4)
    assert list(d["eps"]) == [3, 9, 3] and d["overlay"] is None and np.array_equal(d["rows"][:50], l0)


# ---- whole index directories (need the device index) ----------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("id_type", [np.uint32, np.uint64])
def test_engine_index_directory_decodes(native, orc, c1, tmp_path, id_type):
    import alayalite_amd

    base, _ = c1
    ib = np.dtype(id_type).itemsize
    client = alayalite_amd.Client(str(tmp_path))
    idx = client.create_index("ix", capacity=1200, id_type=id_type)
    idx.fit(base.copy())
    for r in (5, 600):
        idx.remove(r)
    client.save_index("ix")
    d = tmp_path / "ix"
    schema = json.loads((d / "schema.json").read_text())
    assert schema == {"type": "index", "index": {"index_type": "hnsw", "data_type": "float32",
                                                 "id_type": np.dtype(id_type).name, "quantization_type": "none",
                                                 "metric": "l2", "capacity": 1200, "max_nbrs": 32}}
    raw = rf.read_raw(str(d / "raw.data"), ib, np.float32)
    assert (raw["metric"], raw["data_size"], raw["dim"]) == (0, 512, 128)
    assert (raw["item_cnt"], raw["delete_cnt"], raw["capacity"]) == (1000, 2, 1200)
    assert (raw["item_size"], raw["aligned_item_size"], raw["pos"]) == (512, 512, 1000)
    assert np.array_equal(raw["rows"][:1000], base) and not raw["rows"][1000:].any()
    want = np.zeros(1200, bool)
    want[:1000] = True
    want[[5, 600]] = False
    assert np.array_equal(raw["valid"], want)
    g = rf.read_graph(str(d / "hnsw_l2_32.index"), ib)
    assert np.array_equal(g["valid"], want)  # Graph::remove cleared the same bits
    l0 = idx.native().graph_arrays()[0]
    assert np.array_equal(g["rows"][:1000], _ids_as(l0, id_type))


@pytest.mark.gpu
def test_engine_sq8_file_decodes(native, orc, tmp_path):
    import alayalite_amd

    rng = np.random.default_rng(4)
    base = rng.standard_normal((800, 48)).astype(np.float32)
    client = alayalite_amd.Client(str(tmp_path))
    idx = client.create_index("q", capacity=900, quantization_type="sq8", metric="ip")
    idx.fit(base.copy())
    client.save_index("q")
    s = rf.read_sq8(str(tmp_path / "q" / "sq8.data"), 4, np.float32)
    mn, mx = orc.sq8_fit(base)
    assert (s["metric"], s["data_size"], s["dim"], s["item_cnt"], s["capacity"]) == (1, 48, 48, 800, 900)
    assert (s["item_size"], s["aligned_item_size"], s["pos"], s["q_dim"]) == (48, 64, 800, 48)
    assert np.array_equal(s["rows"][:800], orc.sq8_encode(base, mn, mx)) and not s["rows"][800:].any()
    assert np.array_equal(s["min"], mn) and np.array_equal(s["max"], mx)
    assert s["valid"][:800].all() and not s["valid"][800:].any()


def _assemble(tmp_path, name, base, graph, metric_name, metric, id_type, capacity, valid=None, sq8=None):
    l0, levels, off, ue, ep, R = graph
    ib = np.dtype(id_type).itemsize
    wide = (lambda a: _ids_as(a, np.uint64)) if ib == 8 else (lambda a: a)
    d = tmp_path / name
    rf.write_schema(str(d), "hnsw", np.float32, id_type, "sq8" if sq8 is not None else "none", metric_name,
                    capacity, 32)
    rf.write_graph(str(d / f"hnsw_{metric_name}_32.index"), ib, wide(l0), capacity, valid=valid,
                   overlay=(ep, [wide(x) for x in rf.overlay_lists(levels, off, ue, R)]))
    rf.write_raw(str(d / "raw.data"), ib, metric, base, capacity, valid=valid,
                 delete_cnt=0 if valid is None else int((~np.asarray(valid, bool)).sum()))
    if sq8 is not None:
        codes, mn, mx = sq8
        rf.write_sq8(str(d / "sq8.data"), ib, metric, codes, capacity, mn, mx)


@pytest.mark.gpu
@pytest.mark.parametrize("id_type", [np.uint32, np.uint64])
@pytest.mark.parametrize("metric_name,metric", [("l2", 0), ("ip", 1)])
def test_reference_layout_index_loads_and_searches(native, orc, tmp_path, id_type, metric_name, metric):
    """An index directory assembled in the reference's layout (schema.json + graph + raw.data, some
    rows removed) loads through Client(url) and searches exactly like the oracle on the same arrays.
    For 64-bit ids the reference's loader keeps half of each overlay list, and so does the engine."""
    import alayalite_amd

    rng = np.random.default_rng(10 + metric)
    base = rng.standard_normal((1500, 64)).astype(np.float32)
    q = rng.standard_normal((12, 64)).astype(np.float32)
    graph = _oracle_graph(orc, base, metric)
    valid = np.ones(1500, bool)
    valid[[7, 70, 700]] = False
    _assemble(tmp_path, "ref", base, graph, metric_name, metric, id_type, 2000, valid=valid)
    idx = alayalite_amd.Client(str(tmp_path)).get_index("ref")
    ids, dists = idx.batch_search_with_distance(q, 10, 60)
    l0, levels, off, ue, ep, R = graph
    if np.dtype(id_type).itemsize == 8:  # the loaded overlay: first half of each list
        ue = ue.copy()
        for i in np.nonzero(levels)[0]:
            s0, cur = int(off[i]), int(levels[i]) * R
            ue[s0 + cur // 2: s0 + cur] = NONE
    view = orc.IndexView(base, l0, levels, off, ue, R, ep, metric=metric,
                         valid=np.packbits(valid.astype(np.uint8), bitorder="little"))
    for i in range(len(q)):
        r_ids, r_d = view.search(q[i], 10, 60)
        assert np.array_equal(ids[i].astype(np.uint32), r_ids), i
        assert np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32)), i


@pytest.mark.gpu
def test_reference_layout_sq8_index_loads(native, orc, tmp_path):
    """SQ8 index assembled in the reference's layout: batch_search = SQ8 graph search + the
    reference's rerank (index.hpp:337-345, 450-488), equal to the oracle's."""
    import alayalite_amd

    rng = np.random.default_rng(21)
    base = rng.standard_normal((1200, 96)).astype(np.float32)
    q = rng.standard_normal((10, 96)).astype(np.float32)
    graph = _oracle_graph(orc, base, 0)
    mn, mx = orc.sq8_fit(base)
    codes = orc.sq8_encode(base, mn, mx)
    _assemble(tmp_path, "sq", base, graph, "l2", 0, np.uint32, 1200, sq8=(codes, mn, mx))
    idx = alayalite_amd.Client(str(tmp_path)).get_index("sq")
    ids = idx.batch_search(q, 10, 50)
    l0, levels, off, ue, ep, R = graph
    view = orc.IndexView(base, l0, levels, off, ue, R, ep, sq8=(codes, mn, mx, native.host_sq8_order()))
    for i in range(len(q)):
        s_ids, _ = view.search(q[i], 10, 50)
        r_ids, _ = view.rerank(q[i], s_ids, 10, 50)
        assert np.array_equal(ids[i], r_ids), i
