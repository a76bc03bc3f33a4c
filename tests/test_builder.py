"""Host HNSW builder (product) + reference on-disk graph format; checked with the oracle search.

Parity: with one thread the product builder (csrc/hnsw_build.cpp) must produce the reference's
graph exactly -- the oracle's independent restatement of HNSWBuilder::build_graph (oracle_build.cpp,
from hnswlib.hpp:87-751 and hnsw_builder.hpp:98-194), edge for edge, level for level, same entry
point -- including data with massive distance ties (heap order) and degenerate sizes.

Reference coverage restated: python/tests/test_index_types.py:32-80 (recall >= 0.9 on 1k x 128 for
float32/int32/uint32/uint8 data), tests/index/graph_test.cpp:89-130 and hnsw_test.cpp:72-119
(save/load round trip edge by edge)."""

import os

import numpy as np
import pytest


def _view(orc, g, base, metric=0):
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    return orc.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=metric)


def _recall(orc, view, base, queries, k, ef):
    from alayalite_amd.utils import calc_gt, calc_recall

    res = np.stack([view.search(q, k, ef)[0] for q in queries])
    return calc_recall(res, calc_gt(base, queries, k))


def test_builder_structure(native, c1):
    base, _ = c1
    g = native.Graph.build(base, 0, 32, 100, 1, 100)
    l0, levels, off, ue, ep, upper_r, eps = g.arrays()
    assert l0.shape == (1000, 32) and upper_r == 32 and len(eps) == 0
    assert levels[ep] == levels.max()
    for row in l0:
        valid = row[row != 0xFFFFFFFF]
        assert len(valid) == len(set(valid.tolist())) and (valid < 1000).all()
        assert np.all(row[len(valid):] == 0xFFFFFFFF)  # -1 padding after the last edge
    for u in np.nonzero(levels)[0]:
        for lvl in range(1, levels[u] + 1):
            lst = ue[off[u] + (lvl - 1) * 32: off[u] + lvl * 32]
            valid = lst[lst != 0xFFFFFFFF]
            assert len(valid) <= 16 and all(levels[v] >= lvl for v in valid)


def _builder_case(name):
    import zlib

    rng = np.random.default_rng(zlib.crc32(name.encode()))
    metric, R, efc, seed = 0, 32, 100, 100
    if name == "c1":
        base = np.random.default_rng(0).random((1000, 128), dtype=np.float32)
    elif name == "ip96":
        base, metric = rng.standard_normal((800, 96)).astype(np.float32), 1
    elif name == "cos100":
        base = rng.standard_normal((600, 100)).astype(np.float32)
        base /= np.linalg.norm(base, axis=1, keepdims=True)
        metric = 2
    elif name == "int_ties":  # many equal distances: the heaps' tie order decides the edges
        base = rng.integers(0, 4, (1500, 32)).astype(np.float32)
    elif name == "duplicates":
        base = np.repeat(rng.random((200, 24), dtype=np.float32), 4, axis=0)
    elif name == "R16_efc8_seed7":  # ef_construction < M -> ef = M (hnswlib.hpp:104)
        base, R, efc, seed = rng.random((700, 40), dtype=np.float32), 16, 8, 7
    elif name == "R64":
        base, R = rng.random((900, 20), dtype=np.float32), 64
    elif name == "gist_like":
        c = rng.uniform(0, 0.5, (16, 960)).astype(np.float32)
        base = np.clip(c[rng.integers(0, 16, 1200)] + rng.normal(0, 0.05, (1200, 960)), 0, 1).astype(np.float32)
    else:  # tiny sizes
        base = rng.random((int(name[1:]), 8), dtype=np.float32)
    return base, metric, R, efc, seed


@pytest.mark.parametrize("name", ["c1", "ip96", "cos100", "int_ties", "duplicates", "R16_efc8_seed7", "R64",
                                  "gist_like", "n1", "n2", "n17", "n33"])
def test_host_builder_equals_oracle_builder(native, orc, name):
    base, metric, R, efc, seed = _builder_case(name)
    l0, levels, off, ue, ep, upper_r, _ = native.Graph.build(base, metric, R, efc, 1, seed).arrays()
    o_l0, o_levels, o_off, o_ue, o_ep, o_r = orc.build_hnsw(base, metric, R, efc, seed)
    assert np.array_equal(l0, o_l0)
    assert np.array_equal(levels, o_levels) and np.array_equal(off, o_off)
    assert np.array_equal(ue, o_ue)
    assert (ep, upper_r) == (o_ep, o_r)


@pytest.mark.parametrize("kind", ["float64", "int32_wide"])
@pytest.mark.parametrize("metric", [0, 1])
def test_host_builder_generic_order_equals_oracle(native, orc, kind, metric):
    """Non-float DataType (A10): RawSpace<T>::get_distance takes the generic l2_sqr<T>/ip_sqr<T>
    branch (distance_l2.ipp:735-741), so the builder compares rows in that order (metric |
    ALAYA_DIST_GENERIC).  Data whose partial sums are not exact in float, so the order matters."""
    rng = np.random.default_rng(60 + metric)
    if kind == "float64":
        data = rng.standard_normal((700, 50))
    else:
        data = rng.integers(-3000, 3000, (700, 40)).astype(np.int32)
    rows = data.astype(np.float32)
    gen = [orc.lib().orc_l2_generic(orc._ptr(rows[0]), orc._ptr(rows[i]), rows.shape[1], 0) for i in range(1, 40)]
    assert any(np.float32(a) != orc.l2(rows[0], rows[i + 1]) for i, a in enumerate(gen))  # the order is visible
    l0, levels, off, ue, ep, upper_r, _ = native.Graph.build(rows, metric | 0x100, 32, 100, 1, 100).arrays()
    o_l0, o_levels, o_off, o_ue, o_ep, o_r = orc.build_hnsw(rows, metric, 32, 100, 100, generic=True)
    assert np.array_equal(l0, o_l0) and np.array_equal(levels, o_levels)
    assert np.array_equal(ue, o_ue) and (ep, upper_r) == (o_ep, o_r)


def test_single_thread_build_is_deterministic(native, c1):
    base, _ = c1
    a = native.Graph.build(base, 0, 32, 100, 1, 100).arrays()
    b = native.Graph.build(base, 0, 32, 100, 1, 100).arrays()
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.parametrize("threads", [1, 4])
def test_recall_floor_c1(native, orc, c1, threads):
    base, queries = c1
    g = native.Graph.build(base, 0, 32, 100, threads, 100)
    assert _recall(orc, _view(orc, g, base), base, queries, 10, 100) >= 0.9


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.uint8])
def test_recall_floor_int_dtypes(native, orc, dtype):
    rng = np.random.default_rng(5)
    base = rng.integers(0, 100, (1000, 128)).astype(dtype)
    queries = rng.integers(0, 100, (10, 128)).astype(dtype)
    fb, fq = base.astype(np.float32), queries.astype(np.float32)
    g = native.Graph.build(fb, 0, 32, 100, 1, 100)
    assert _recall(orc, _view(orc, g, fb), fb, fq, 10, 100) >= 0.9


def test_graph_file_round_trip(native, c1, tmp_path):
    base, _ = c1
    g = native.Graph.build(base, 0, 32, 100, 1, 100)
    path = str(tmp_path / "hnsw_l2_32.index")
    g.save(path, 4, 100000)
    # reference layout: capacity rows of 128 B + bitmap + overlay section
    assert os.path.getsize(path) > 100000 * 128
    h = native.Graph.load(path, 4)
    for x, y in zip(g.arrays(), h.arrays()):
        assert np.array_equal(np.asarray(x), np.asarray(y))


def test_graph_file_round_trip_u64(native, c1, tmp_path):
    base, _ = c1
    g = native.Graph.build(base[:300], 0, 32, 100, 1, 100)
    path = str(tmp_path / "g64.index")
    g.save(path, 8, 300)
    h = native.Graph.load(path, 8)
    assert np.array_equal(g.arrays()[0], h.arrays()[0])


def test_nsg_style_graph_import(native):
    l0 = np.full((4, 32), 0xFFFFFFFF, np.uint32)
    l0[0, :2] = [1, 2]
    g = native.Graph.from_arrays(l0, None, None, None, 0, 0, np.array([0, 3], np.uint32))
    assert list(g.arrays()[-1]) == [0, 3]
