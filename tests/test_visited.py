"""The visited set's second level (DynamicBitset semantics, include/utils/query_utils.hpp:69-115):
a query whose LDS table fills spills to a per-slot global bitset that is clean between queries --
the spilling query zeroes only the words it set (its dirty list), or the whole bitset when the list
overflows.  Every case runs the batch twice: a word left set by one query would mark rows visited
for a later query on the same slot and change its ids, distances or counters."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(view, ids, dists, cnt, queries, k, ef, sq8=False):
    for i, q in enumerate(queries):
        r_ids, r_d, r_c = view.search(q, k, ef, with_counters=True)
        assert np.array_equal(ids[i], r_ids), (i, ids[i], r_ids)
        assert np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32)), i
        assert tuple(cnt[i]) == tuple(r_c), (i, cnt[i], r_c)


@pytest.mark.parametrize("dirty_cap", [None, "3"])
def test_spilled_slots_are_left_clean(native, orc, monkeypatch, dirty_cap):
    """64-slot tables (every query spills at once) over 300 queries on a few slots, twice; with a
    3-word dirty list every query takes the whole-bitset clearing fallback."""
    if dirty_cap:
        monkeypatch.setenv("ALAYA_DIRTY_CAP", dirty_cap)
    rng = np.random.default_rng(40)
    base = rng.random((20000, 24), dtype=np.float32)
    queries = rng.random((300, 24), dtype=np.float32)
    g = native.Graph.build(base, 0, 32, 100, 8, 100)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    dev.set_hash_log2(6)
    dev.set_visited_mode(1)
    first = dev.search(queries, 10, 120)
    second = dev.search(queries[::-1].copy(), 10, 120)
    _check(view, *first, queries, 10, 120)
    _check(view, *second, queries[::-1], 10, 120)


def _circulant_graph(n, R, seed):
    """Row i links to (i + c_j) mod n for R distinct nonzero offsets c_j: no self loops, no repeated
    ids in a row, every row full.  Built in O(n R) numpy (no HNSW build at 10M rows)."""
    rng = np.random.default_rng(seed)
    c = rng.choice(np.arange(1, n, dtype=np.int64), R, replace=False)
    rows = np.arange(n, dtype=np.int64)[:, None]
    return ((rows + c[None, :]) % n).astype(np.uint32)


@pytest.mark.parametrize("waves", ["1", "4"])
def test_sq8_spill_at_10m_rows(native, orc, monkeypatch, waves):
    """Config 5's id width: 10M rows (24-bit ids, 1.25 MB bitset per slot), SQ8 IP search plus the
    reference rerank, tables forced to 1024 slots so every query spills; searchers packed 1 or 4 per
    workgroup (the SQ8 layout shares the quantizer's scale / min per workgroup).  Rows are 32-d so
    the base fits a test (1.3 GB); the graph is circulant (no overlay: NSG-style entry points)."""
    monkeypatch.setenv("ALAYA_SEARCH_WAVES", waves)
    n, d, k, ef = 10_000_000, 32, 10, 48
    rng = np.random.default_rng(77)
    base = rng.standard_normal((n, d), dtype=np.float32)
    queries = rng.standard_normal((13, d), dtype=np.float32)
    l0 = _circulant_graph(n, 32, 5)
    eps = np.array([0], np.uint32)  # one NSG-style entry point (the restatement's no-overlay path)
    g = native.Graph.from_arrays(l0, None, None, None, 0, 0, eps)
    mn, mx = native.sq8_train(base)
    codes = native.sq8_encode(base, mn, mx, 16)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 1)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    dev.set_hash_log2(10)
    view = orc.IndexView(base, l0, None, None, None, 0, 0, metric=1, sq8=(codes, mn, mx, 2))
    for rep in range(2):
        s_ids, s_d, s_c = dev.search_sq8(queries, k, ef, 0)
        r_ids, r_d, _ = dev.search_sq8(queries, k, ef, 1)
        for i, q in enumerate(queries):
            o_ids, o_d, o_c = view.search(q, k, ef, with_counters=True)
            assert np.array_equal(s_ids[i], o_ids), (rep, i)
            assert np.array_equal(s_d[i].view(np.uint32), o_d.view(np.uint32)), (rep, i)
            assert tuple(s_c[i]) == tuple(o_c), (rep, i, s_c[i], o_c)
            rr_ids, rr_d = view.rerank(q, o_ids, k, ef)
            assert np.array_equal(r_ids[i], rr_ids), (rep, i)
            assert np.array_equal(r_d[i].view(np.uint32), rr_d.view(np.uint32)), (rep, i)
        assert s_c[:, 0].min() > 1000  # n_dist: far past the 1024-slot table's ~700 entries


@pytest.mark.parametrize("waves", ["1", "2", "4"])
@pytest.mark.parametrize("nq", [1, 5, 64, 301])
def test_sq8_searchers_per_workgroup(native, orc, monkeypatch, waves, nq):
    """1, 2 or 4 SQ8 searchers per workgroup (shared scale / min), batch sizes that do not fill the
    last workgroup: ids, distance bits and counters equal the restatement's."""
    monkeypatch.setenv("ALAYA_SEARCH_WAVES", waves)
    rng = np.random.default_rng(nq)
    base = rng.standard_normal((3000, 768)).astype(np.float32)
    queries = rng.standard_normal((nq, 768)).astype(np.float32)
    g = native.Graph.build(base, 1, 32, 100, 8, 100)
    mn, mx = native.sq8_train(base)
    codes = native.sq8_encode(base, mn, mx, 8)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=1, sq8=(codes, mn, mx, 2))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 1)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    ids, d, c = dev.search_sq8(queries, 10, 64, 0)
    _check(view, ids, d, c, queries, 10, 64)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("pct", ["50", "95", "100"])
def test_spill_threshold_keeps_results_exact(native, orc, monkeypatch, mode, pct):
    """The first-level spill threshold (ALAYA_VIS_LIMIT_PCT, clamped to slots - 64) only moves the
    point where a query starts using the second level: compact and wide 256-slot tables filled to
    any threshold return the restatement's ids, distance bits and counters."""
    monkeypatch.setenv("ALAYA_VIS_LIMIT_PCT", pct)
    rng = np.random.default_rng(41)
    base = rng.random((6000, 24), dtype=np.float32)
    queries = rng.random((80, 24), dtype=np.float32)
    g = native.Graph.build(base, 0, 32, 100, 8, 100)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    dev.set_hash_log2(8)
    dev.set_visited_mode(mode)
    _check(view, *dev.search(queries, 10, 150), queries, 10, 150)

