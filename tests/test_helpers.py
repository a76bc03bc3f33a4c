"""Distance helpers (search kernel kMode 4): waves with no query left compute a sibling's predicted
next expansion into an LDS memo that the sibling reads.

The bar is the same as every search test: ids, distance bits and counters equal the restatement
(graph_search_job.hpp:221-371, query_utils.hpp:69-115 / 236-312).  Small batches put one searcher
and three helpers in most workgroups from the first expansion (the grid fills the CUs whatever the
batch), so nearly every expansion of every query is helped; a batch larger than the resident
searchers runs the first round statically and the rest from the work counter, and its tail is
helped.  help_stats() reports how many fresh distances came from a memo, so the tests also check
that the memo path really ran.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _graph_view(native, orc, base, metric=0, threads=8, valid=None):
    g = native.Graph.build(base, metric, 32, 100, threads, 100)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    return g, orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, valid=valid)


def _check(view, ids, dists, cnt, queries, k, ef, rows=None):
    for i in (range(len(queries)) if rows is None else rows):
        r_ids, r_d, r_c = view.search(queries[i], k, ef, with_counters=True)
        assert np.array_equal(ids[i], r_ids), (i, ids[i], r_ids)
        assert np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32)), (i, dists[i], r_d)
        assert tuple(cnt[i]) == tuple(r_c), (i, cnt[i], r_c)


@pytest.fixture(scope="module")
def sift_like(native, orc):
    rng = np.random.default_rng(55)
    base = rng.integers(0, 128, (20000, 128)).astype(np.float32)
    queries = rng.integers(0, 128, (5000, 128)).astype(np.float32)
    g, view = _graph_view(native, orc, base)
    return base, queries, g, view


@pytest.mark.parametrize("hint", ["1", "2"])
@pytest.mark.parametrize("ef", [40, 128])
def test_helped_small_batches_bit_exact(native, sift_like, monkeypatch, ef, hint):
    """d = 128 L2 (the SIFT kernel), batches of 1 .. 600 queries: most workgroups run one searcher
    and three helpers.  ALAYA_HELP_FLAGS (search_kernels.hip, help_siblings): bit 0 forces the
    visited hint off, bit 1 forces it on.  "1": helpers compute every claimed row (the f32 default);
    "2": they first look each id up in the sibling's LDS table (table_lookup<true>)."""
    base, queries, g, view = sift_like
    monkeypatch.setenv("ALAYA_HELP_FLAGS", hint)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    dev.set_helpers(1)
    memo = own = 0
    for nq in (1, 7, 64, 600):
        for rep in range(2):  # twice on the same slots
            ids, dists, cnt = dev.search(queries[:nq], 10, ef)
            m, x, _ = dev.help_stats()
            assert x <= int(cnt[:, 1].sum())
            memo, own = memo + m, own + int(cnt[:, 0].sum()) - m
            assert m <= int(cnt[:, 0].sum()), (nq, rep, m)
            _check(view, ids, dists, cnt, queries[:nq], 10, ef)
    assert memo > 0, (memo, own)


def test_helped_large_batch_tail(native, sift_like):
    """5000 queries > the resident searchers: the first round is assigned statically, the rest come
    from the work counter (offset past the first round), and the batch tail is helped."""
    base, queries, g, view = sift_like
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    dev.set_helpers(0)
    ids0, d0, c0 = dev.search(queries, 10, 64)
    dev.set_helpers(1)
    ids, dists, cnt = dev.search(queries, 10, 64)
    assert dev.help_stats()[0] <= int(cnt[:, 0].sum())
    assert np.array_equal(ids, ids0) and np.array_equal(dists.view(np.uint32), d0.view(np.uint32))
    assert np.array_equal(cnt, c0)
    _check(view, ids, dists, cnt, queries, 10, 64, rows=range(0, 5000, 97))


@pytest.mark.parametrize("metric", [1, 0])
def test_helped_d256_and_invalid_rows(native, orc, monkeypatch, metric):
    """d = 256 (8 chunks), IP and L2, with rows cleared in the validity bitmap (FLT_MAX from the
    memo as from the searcher, raw_space.hpp:298-300)."""
    rng = np.random.default_rng(77 + metric)
    base = rng.standard_normal((8000, 256)).astype(np.float32)
    queries = rng.standard_normal((40, 256)).astype(np.float32)
    valid = np.full(8000 // 8, 0xFF, np.uint8)
    valid[::7] = 0x5A
    g, view = _graph_view(native, orc, base, metric=metric, valid=valid)
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric, valid)
    dev.set_graph(g)
    dev.set_helpers(1)
    for nq in (3, 40):
        ids, dists, cnt = dev.search(queries[:nq], 10, 96)
        _check(view, ids, dists, cnt, queries[:nq], 10, 96)


N8 = 20_000


@pytest.fixture(scope="module")
def sq8_setups(native, orc):
    cache = {}

    def get(metric):
        if metric not in cache:
            d = 768
            rng = np.random.default_rng(4000 + metric)
            centres = rng.standard_normal((64, d)).astype(np.float32)
            base = (centres[rng.integers(0, 64, N8)] + 0.35 * rng.standard_normal((N8, d))).astype(np.float32)
            queries = (centres[rng.integers(0, 64, 24)] + 0.35 * rng.standard_normal((24, d))).astype(np.float32)
            g = native.Graph.build(base, metric, 32, 100, 8, 100)
            mn, mx = native.sq8_train(base)
            codes = native.sq8_encode(base, mn, mx, 8)
            l0, levels, off, ue, ep, ur, _ = g.arrays()
            view = orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, sq8=(codes, mn, mx, 2))
            cache[metric] = (base, queries, g, mn, mx, codes, view)
        return cache[metric]

    return get


@pytest.mark.parametrize("ef", [40, 340])
@pytest.mark.parametrize("metric", [1, 0])
def test_helped_sq8_768_spilled(native, sq8_setups, metric, ef):
    """Config 5's kernel (768-d SQ8, AVX-512 order, spill table): a 128-slot first level spills at
    the first expansion, helpers read the sibling's spill-table buckets for their visited hint;
    search ids / distance bits / counters and the reference rerank equal the restatement."""
    base, queries, g, mn, mx, codes, view = sq8_setups(metric)
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    dev.set_hash_log2(7)
    dev.set_helpers(1)
    memo = 0
    for nq in (1, 5, 24):
        qs = queries[:nq]
        for rep in range(2):
            s_ids, s_d, s_c = dev.search_sq8(qs, 10, ef, 0)
            memo += dev.help_stats()[0]
            r_ids, r_d, _ = dev.search_sq8(qs, 10, ef, 1)
            for i, q in enumerate(qs):
                o_ids, o_d, o_c = view.search(q, 10, ef, with_counters=True)
                assert np.array_equal(s_ids[i], o_ids), (nq, rep, i)
                assert np.array_equal(s_d[i].view(np.uint32), o_d.view(np.uint32)), (nq, rep, i)
                assert tuple(s_c[i]) == tuple(o_c), (nq, rep, i, s_c[i], o_c)
                rr = view.rerank(q, o_ids, 10, ef)
                assert np.array_equal(r_ids[i], rr[0]) and np.array_equal(r_d[i].view(np.uint32), rr[1].view(np.uint32))
    assert memo > 0


@pytest.mark.parametrize("ef", [12, 40])
@pytest.mark.parametrize("metric", [1, 0])
def test_helped_sq8_128_memo_over_the_table(native, orc, metric, ef):
    """SQ8 d = 128 (AVX-512 order, spill table, helpers and the visited hint on by default): the
    query region (512 B) is smaller than the memo (4 x 2 x 32 x 8 B), so the memo overlays the memo
    wave's pool and visited table (memo_off > 0).  A wave that runs out of queries retires its
    requests and sets its helper bit before it clears that area, and the hint's probe of a
    sibling's wide table is bounded: batches of 1 .. 64 queries at small ef, where the
    zeroed table would once have made a helper's probe spin, finish with the restatement's ids,
    distance bits and counters."""
    d, n = 128, 6000
    rng = np.random.default_rng(910 + metric)
    base = rng.standard_normal((n, d)).astype(np.float32)
    queries = rng.standard_normal((64, d)).astype(np.float32)
    g = native.Graph.build(base, metric, 32, 100, 8, 100)
    mn, mx = native.sq8_train(base)
    codes = native.sq8_encode(base, mn, mx, 8)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, sq8=(codes, mn, mx, 2))
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    dev.set_helpers(1)
    for nq in (1, 5, 64):
        qs = queries[:nq]
        for rep in range(2):
            s_ids, s_d, s_c = dev.search_sq8(qs, 10, ef, 0)
            for i, q in enumerate(qs):
                o_ids, o_d, o_c = view.search(q, 10, ef, with_counters=True)
                assert np.array_equal(s_ids[i], o_ids), (nq, rep, i)
                assert np.array_equal(s_d[i].view(np.uint32), o_d.view(np.uint32)), (nq, rep, i)
                assert tuple(s_c[i]) == tuple(o_c), (nq, rep, i, s_c[i], o_c)
