"""The fixed-d SQ8 kernels that config 5 runs (d = 768: 24 chunks of 32 codes, d = 960: 30), forced
into their spilled visited regime.

A 128-slot first-level table (set_hash_log2(7)) spills after ~25 ids (a 256-slot one after ~110),
so every query spends almost all of its expansions on the second level, as config 5's 10k-query
batch does (355 of 385 expansions per query): the spilled visit path with the next expansion's
second-level state read one expansion ahead, and the per-slot cleanup at the query's end.  Both SQ8
reduction orders (AVX-512: 2, AVX2: 1), L2 and IP, 1 or 4 searchers per workgroup, ef 40 and 340.
Every batch runs twice on the same slots (a slot left dirty by one query would change a later one's
ids, distances or counters), and ids, distance bits and counters must equal the restatement's
search (graph_search_job.hpp:237-251, query_utils.hpp:69-115, distance_ip.ipp:292-366 /
distance_l2.ipp:334-408); the reference rerank (index.hpp:337-345, 450-488) must equal view.rerank.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 20_000
NQ = 24
K = 10


@pytest.fixture(scope="module")
def setups(native, orc):
    """One host-built graph per (d, metric), shared by the cases (SQ8 codes per reduction order)."""
    cache = {}

    def get(d, metric, order):
        key = (d, metric)
        if key not in cache:
            rng = np.random.default_rng(1000 + d + metric)
            centres = rng.standard_normal((64, d)).astype(np.float32)
            base = (centres[rng.integers(0, 64, N)] + 0.35 * rng.standard_normal((N, d))).astype(np.float32)
            queries = (centres[rng.integers(0, 64, NQ)] + 0.35 * rng.standard_normal((NQ, d))).astype(np.float32)
            g = native.Graph.build(base, metric, 32, 100, 8, 100)
            mn, mx = native.sq8_train(base)
            codes = native.sq8_encode(base, mn, mx, 8)
            cache[key] = (base, queries, g, mn, mx, codes)
        base, queries, g, mn, mx, codes = cache[key]
        l0, levels, off, ue, ep, ur, _ = g.arrays()
        view = orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, sq8=(codes, mn, mx, order))
        return base, queries, g, mn, mx, codes, view

    return get


def _run(native, setup, order, metric, ef, visited_mode=0, log2_slots=7):
    base, queries, g, mn, mx, codes, view = setup
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, order)
    dev.set_hash_log2(log2_slots)
    dev.set_visited_mode(visited_mode)
    expect = [view.search(q, K, ef, with_counters=True) for q in queries]
    rerank = [view.rerank(q, e[0], K, ef) for q, e in zip(queries, expect)]
    for rep in range(2):
        qs = queries if rep == 0 else queries[::-1].copy()
        ex = expect if rep == 0 else expect[::-1]
        rr = rerank if rep == 0 else rerank[::-1]
        s_ids, s_d, s_c = dev.search_sq8(qs, K, ef, 0)
        r_ids, r_d, _ = dev.search_sq8(qs, K, ef, 1)
        for i in range(len(qs)):
            o_ids, o_d, o_c = ex[i]
            assert np.array_equal(s_ids[i], o_ids), (rep, i, s_ids[i], o_ids)
            assert np.array_equal(s_d[i].view(np.uint32), o_d.view(np.uint32)), (rep, i)
            assert tuple(s_c[i]) == tuple(o_c), (rep, i, s_c[i], o_c)
            assert np.array_equal(r_ids[i], rr[i][0]), (rep, i, r_ids[i], rr[i][0])
            assert np.array_equal(r_d[i].view(np.uint32), rr[i][1].view(np.uint32)), (rep, i)
        # far past the ids the first level holds before it spills (~25 with 128 slots; the
        # multi-threaded host build varies the graph, so the margin is generous)
        assert s_c[:, 0].min() > 100, s_c[:, 0].min()


@pytest.mark.parametrize("ef", [40, 340])
@pytest.mark.parametrize("waves", ["1", "4"])
@pytest.mark.parametrize("order", [2, 1])
@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("d", [768, 960])
def test_fixed_d_sq8_spilled_bit_exact(native, setups, monkeypatch, d, metric, order, waves, ef):
    monkeypatch.setenv("ALAYA_SEARCH_WAVES", waves)
    _run(native, setups(d, metric, order), order, metric, ef)


@pytest.mark.parametrize("spill_table", [None, "0", "6", "9"])
@pytest.mark.parametrize("visited_mode", [1, 2])
@pytest.mark.parametrize("dirty_cap", [None, "3"])
def test_fixed_d_sq8_spilled_second_levels(native, setups, monkeypatch, spill_table, visited_mode, dirty_cap):
    """Config 5's kernel (768-d IP, AVX-512 order, 4 searchers per workgroup) on each second level:
    the spill table at its default size (2^14 entries per slot), the N-bit bitset
    (ALAYA_SPILL_TABLE=0), and tables of 64 / 512 entries whose buckets fill up, so many ids take
    the bitset third level; compact and wide first-level tables (flushed into the spill table when
    the query spills); a 3-entry dirty list, so a query that used the bitset takes the whole-bitset
    cleanup fallback."""
    monkeypatch.setenv("ALAYA_SEARCH_WAVES", "4")
    if dirty_cap:
        monkeypatch.setenv("ALAYA_DIRTY_CAP", dirty_cap)
    if spill_table is not None:
        monkeypatch.setenv("ALAYA_SPILL_TABLE", spill_table)
    _run(native, setups(768, 1, 2), 2, 1, 340, visited_mode, 8)


@pytest.mark.parametrize("ef", [40, 340])
@pytest.mark.parametrize("waves", ["1", "4"])
@pytest.mark.parametrize("metric", [1, 0])
@pytest.mark.parametrize("d", [768, 960])
def test_spill_table_prefetch_matches_a_reread(native, setups, monkeypatch, d, metric, waves, ef):
    """The order the spill-table prefetch relies on, checked at run time: ALAYA_SPILL_FLAGS bit 8 runs
    the kDiag = 2 kernel, which re-reads every bucket it read one expansion ahead, at the visit that
    uses it (after a workgroup fence and s_waitcnt(0)), and sets bit 30 of the query's n_hops_upper
    counter when any differs -- so a stale prefetch (a bucket read before the previous visit's
    stores landed) fails the counter comparison with the restatement."""
    monkeypatch.setenv("ALAYA_SEARCH_WAVES", waves)
    monkeypatch.setenv("ALAYA_SPILL_FLAGS", "256")
    _run(native, setups(d, metric, 2), 2, metric, ef)
