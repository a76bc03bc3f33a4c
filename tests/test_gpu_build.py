"""Device HNSW construction (alaya_index_build_graph, the GPU analogue of HNSWBuilder::build_graph,
include/index/graph/hnsw/hnsw_builder.hpp:98-194 over hnswlib add_point, hnswlib.hpp:652-751).

The device build is batched insertion, so its graph is not the sequential one; what is pinned:
  * structure: level-0 rows hold <= R distinct ids != self, -1 only as trailing padding; upper
    lists hold <= R/2 ids of nodes that exist on that level; levels are exactly the reference's
    draw (same seeded engine as the host builder); the entry point is a node of the top level;
  * determinism: two builds of the same rows give the same graph;
  * quality: the reference's recall floors (python/tests/test_index_types.py:32-80, >= 0.9 on
    1k x 128 at ef 100) for L2 / IP / COS, and recall within 0.02 of the host-built graph;
  * the graph installed on the device and its host copy search identically, and both match the
    CPU restatement of the search (oracle/) bit for bit."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(n, nq, d, seed):
    rng = np.random.default_rng(seed)
    return rng.random((n, d), dtype=np.float32), rng.random((nq, d), dtype=np.float32)


def _normalize(x):
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def _gt(base, q, k, metric):
    b = base.astype(np.float64)
    out = []
    for v in q.astype(np.float64):
        d = ((b - v) ** 2).sum(1) if metric == 0 else -(b @ v)
        out.append(np.argsort(d, kind="stable")[:k])
    return np.array(out)


def _recall(ids, gt):
    return np.mean([len(set(a.tolist()) & set(b.tolist())) / len(b) for a, b in zip(ids, gt)])


def _build(native, base, metric=0, R=32, efc=100, batch_div=0, max_batch=0, refine=1):
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric, None)
    g, stats = dev.build_graph(R, efc, 100, batch_div, max_batch, refine)
    return dev, g, stats


def _check_structure(g, n, R):
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    assert l0.shape == (n, R) and upper_r == R
    for i in range(n):
        row = l0[i]
        cnt = int(np.argmax(row == 0xFFFFFFFF)) if (row == 0xFFFFFFFF).any() else R
        assert (row[cnt:] == 0xFFFFFFFF).all(), i
        live = row[:cnt]
        assert (live < n).all() and i not in live and len(set(live.tolist())) == cnt, i
    top = int(levels.max())
    assert levels[ep] == top
    for i in np.nonzero(levels)[0]:
        for lv in range(1, int(levels[i]) + 1):
            lst = ue[off[i] + (lv - 1) * R: off[i] + lv * R]
            live = lst[lst != 0xFFFFFFFF]
            assert len(live) <= R // 2 and (lst[len(live):] == 0xFFFFFFFF).all()
            assert i not in live and all(levels[v] >= lv for v in live), (i, lv)
    return l0, levels


def test_structure_levels_and_determinism(native):
    base, _ = _data(4000, 1, 48, 11)
    _, g1, st = _build(native, base)
    l0, levels = _check_structure(g1, 4000, 32)
    host = native.Graph.build(base, 0, 32, 100, 1, 100)
    assert np.array_equal(levels, host.arrays()[1])  # same seeded level draw as the reference
    assert st["batches"] > 10 and st["max_level"] == int(levels.max())
    _, g2, _ = _build(native, base)
    for a, b in zip(g1.arrays(), g2.arrays()):
        if isinstance(a, np.ndarray):
            assert np.array_equal(a, b)
        else:
            assert a == b


@pytest.mark.parametrize("metric", [0, 1, 2])
def test_recall_floor_c1_shape(native, metric):
    """test_index_types.py:32-80: 1k x 128, recall@10 >= 0.9 at ef 100 (reference floor)."""
    base, q = _data(1000, 100, 128, 0)
    if metric == 2:  # COS indexes store normalised rows (raw_space.hpp:131-140)
        base, q = _normalize(base), _normalize(q)
    dev, _, _ = _build(native, base, metric=1 if metric == 2 else metric)
    ids, _, _ = dev.search(q, 10, 100)
    assert _recall(ids, _gt(base, q, 10, 0 if metric == 0 else 1)) >= 0.9


def test_recall_close_to_host_build(native):
    """20k x 64: recall@10 at ef in {16, 32, 64} within 0.02 of the host-built graph (16 threads)."""
    base, q = _data(20000, 200, 64, 3)
    gt = _gt(base, q, 10, 0)
    dev, _, _ = _build(native, base)
    host = native.DeviceIndex(0)
    host.set_base(base, 0, None)
    host.set_graph(native.Graph.build(base, 0, 32, 100, 16, 100))
    for ef in (16, 32, 64):
        r_dev = _recall(dev.search(q, 10, ef)[0], gt)
        r_host = _recall(host.search(q, 10, ef)[0], gt)
        assert r_dev >= r_host - 0.02, (ef, r_dev, r_host)


def test_installed_graph_equals_host_copy_and_oracle(native, orc):
    base, q = _data(3000, 40, 96, 5)
    dev, g, _ = _build(native, base)
    ids, dists, cnt = dev.search(q, 10, 50)
    other = native.DeviceIndex(0)
    other.set_base(base, 0, None)
    other.set_graph(g)
    ids2, dists2, cnt2 = other.search(q, 10, 50)
    assert np.array_equal(ids, ids2) and np.array_equal(dists.view(np.uint32), dists2.view(np.uint32))
    assert np.array_equal(cnt, cnt2)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=0)
    for i in range(q.shape[0]):
        r_ids, r_d, r_c = view.search(q[i], 10, 50, with_counters=True)
        assert np.array_equal(ids[i], r_ids) and np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32))
        assert tuple(cnt[i]) == tuple(r_c)


@pytest.mark.parametrize("dim,n", [(24, 1500), (960, 600)])
def test_single_point_batches_reproduce_the_sequential_build(native, orc, dim, n):
    """batch_div = max_batch = 1, no refine: points are inserted one at a time in label order, which
    is the reference's sequential add_point (num_threads = 1).  On tie-free data the device graph
    equals the oracle's restatement of HNSWBuilder::build_graph exactly (oracle_build.cpp from
    hnswlib.hpp:652-751), and so the product's host build too."""
    base, _ = _data(n, 1, dim, 17)
    for metric in (0, 1):
        _, g, st = _build(native, base, metric=metric, batch_div=1, max_batch=1, refine=0)
        assert st["max_batch"] == 1
        l0, levels, off, ue, ep, upper_r, _ = g.arrays()
        o_l0, o_levels, o_off, o_ue, o_ep, o_r = orc.build_hnsw(base, metric, 32, 100, 100)
        assert np.array_equal(l0, o_l0) and np.array_equal(levels, o_levels)
        assert np.array_equal(off, o_off) and np.array_equal(ue, o_ue) and (ep, upper_r) == (o_ep, o_r)


@pytest.mark.parametrize("batch_div,max_batch", [(1, 1), (2, 64), (64, 0)])
def test_batch_schedules(native, batch_div, max_batch):
    """batch of one point (sequential insertion order), tiny batches, very small batches."""
    base, q = _data(1500, 50, 32, 9)
    dev, g, st = _build(native, base, batch_div=batch_div, max_batch=max_batch)
    _check_structure(g, 1500, 32)
    if max_batch == 1:
        assert st["max_batch"] == 1
    ids, _, _ = dev.search(q, 10, 64)
    assert _recall(ids, _gt(base, q, 10, 0)) >= 0.9


def test_index_fit_gpu_builder(native):
    import alayalite_amd as al

    base, q = _data(2000, 30, 64, 21)
    idx = al.Index("g", al.IndexParams(metric="l2"))
    idx.fit(base, ef_construction=100, num_threads=1, builder="gpu")
    ids = idx.batch_search(q, 10, 64)
    assert _recall(ids, _gt(base, q, 10, 0)) >= 0.9
    with pytest.raises(ValueError):
        al.Index("h").fit(base, builder="cpu")


def test_small_and_degenerate(native):
    for n in (1, 2, 3, 40):
        base, q = _data(n, 3, 16, n)
        dev, g, _ = _build(native, base)
        _check_structure(g, n, 32)
        ids, _, _ = dev.search(q, 1, 10)
        assert (ids < n).all()
    # duplicate rows (zero distances everywhere)
    base = np.ones((500, 8), np.float32)
    dev, g, _ = _build(native, base)
    _check_structure(g, 500, 32)
