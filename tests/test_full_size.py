"""Parity at the benchmark configurations' full sizes, inside the GPU suite.

The bench's CPU leg checks the headline (GIST 1M, 1k queries) on every driver run; these tests pin
the other single-GPU configurations the same way, at their full index and batch sizes, so that the
paths only those shapes take are checked where they run:
  * config 3, SIFT-shaped 1M x 128 L2, a 10k-query batch at ef 70 -- more queries than resident
    searchers, so the batch's last queries run beside distance helpers (search_kernels.hip,
    help_siblings) and the two-waves policy stays off;
  * config 4, GIST-shaped 1M x 960 L2 at ef 373: the 10k batch (one wave per SIMD) and a rank's
    1,250-query group of the S = 1 layout (two waves per SIMD, kMode 8);
  * config 5, 10M x 768 IP with SQ8 search + the reference rerank, 10k queries at ef 368 -- the
    spill-table second level at its real table size, with helpers.
The whole batch runs on the device in one launch; a sample of its queries (spread over the batch,
plus the last ones, which finish in the tail) is compared with the CPU restatement (oracle/)
searching the same device-built graph: ids, distance bits and traversal counters
(graph_search_job.hpp:221-371), and for config 5 the reranked ids and distances
(index.hpp:337-345, 450-488)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 10


def _sample(nq, spread=240, tail=60):
    return np.unique(np.concatenate([np.linspace(0, nq - 1, spread).astype(np.int64), np.arange(nq - tail, nq)]))


def _view(orc, g, base, metric=0, sq8=None):
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    return orc.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=metric, sq8=sq8)


def _check(view, queries, ids, dists, cnt, ef, sample):
    for i in sample:
        o_ids, o_d, o_c = view.search(queries[i], K, ef, with_counters=True)
        assert np.array_equal(ids[i], o_ids), (i, ids[i], o_ids)
        assert np.array_equal(dists[i].view(np.uint32), o_d.view(np.uint32)), i
        assert tuple(int(x) for x in cnt[i]) == tuple(int(x) for x in o_c), (i, cnt[i], o_c)


def test_config3_sift_1m_10k_batch(native, orc):
    from workloads.datasets import sift_like

    base, queries = sift_like(1_000_000, 10_000)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    g, _ = dev.build_graph(32, 100, 100, 0, 0, 2)
    ids, dists, cnt = dev.search(queries, K, 70)
    view = _view(orc, g, base)
    _check(view, queries, ids, dists, cnt, 70, _sample(len(queries)))
    hits, _, rows = dev.help_stats()
    assert rows > 0, "a 10k batch past the resident searchers should run with helpers"


@pytest.fixture(scope="module")
def gist1m(native):
    from workloads.datasets import gist_like

    base, queries = gist_like(1_000_000, 10_000)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    g, _ = dev.build_graph(32, 100, 100, 0, 0, 2)
    return base, queries, dev, g


@pytest.mark.parametrize("nq", [10_000, 1_250])
def test_config4_gist_1m(native, orc, gist1m, nq):
    base, queries, dev, g = gist1m
    qs = np.ascontiguousarray(queries[:nq])
    ids, dists, cnt = dev.search(qs, K, 373)
    grid, waves = dev.last_launch()
    if nq == 1_250:  # past 1,024 resident one-wave searchers, below 1.5x: the two-waves kernel
        assert grid * waves >= 1_250, (grid, waves)  # (the grid is capped at the batch)
    view = _view(orc, g, base)
    _check(view, qs, ids, dists, cnt, 373, _sample(nq, spread=120, tail=30))


def test_config5_sq8_10m_10k_batch(native, orc):
    from workloads.datasets import text_like

    base, queries = text_like(10_000_000, 10_000)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 1)
    g, _ = dev.build_graph(32, 100, 100, 0, 0, 2)
    mn, mx = native.sq8_train(base)
    codes = native.sq8_encode(base, mn, mx, 16)
    order = native.host_sq8_order()
    dev.set_sq8(codes, mn, mx, order)
    ef = 368
    s_ids, s_d, s_c = dev.search_sq8(queries, K, ef, 0)
    r_ids, r_d, _ = dev.search_sq8(queries, K, ef, 1)
    view = _view(orc, g, base, metric=1, sq8=(codes, mn, mx, order))
    sample = _sample(len(queries), spread=100, tail=30)
    _check(view, queries, s_ids, s_d, s_c, ef, sample)
    for i in sample:
        o_ids, o_d = view.rerank(queries[i], s_ids[i], K, ef)
        assert np.array_equal(r_ids[i], o_ids), (i, r_ids[i], o_ids)
        assert np.array_equal(r_d[i].view(np.uint32), o_d.view(np.uint32)), i
