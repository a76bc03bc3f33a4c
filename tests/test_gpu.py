"""Device parity: the HIP path (through the C ABI) against the CPU restatement, bit for bit.

Bar: integer/index outputs (neighbour ids, counters) identical; float distances identical in
their bit pattern (the device reproduces the reference's AVX2 reduction order exactly)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _graph_view(native, orc, base, metric=0, threads=1, R=32, valid=None):
    g = native.Graph.build(base, metric, R, 100, threads, 100)
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=metric, valid=valid)
    return g, view


def _dev(native, base, g, metric=0, valid=None):
    d = native.DeviceIndex(0)
    d.set_base(base, metric, valid)
    d.set_graph(g)
    return d


def _check(view, dev, queries, k, ef):
    ids, dists, cnt = dev.search(queries, k, ef)
    for i, q in enumerate(queries):
        r_ids, r_d, r_c = view.search(q, k, ef, with_counters=True)
        assert np.array_equal(ids[i], r_ids), (i, ids[i], r_ids)
        assert np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32)), (i, dists[i], r_d)
        assert tuple(cnt[i]) == tuple(r_c), (i, cnt[i], r_c)
    return ids


@pytest.mark.parametrize("dim", [1, 2, 5, 8, 13, 16, 24, 31, 32, 33, 40, 64, 96, 100, 127, 128, 129,
                                 200, 255, 256, 384, 512, 768, 800, 960, 1000, 1024])
@pytest.mark.parametrize("metric", [0, 1])
def test_distance_kernel_bit_exact(native, orc, dim, metric):
    rng = np.random.default_rng(dim * 7 + metric)
    base = rng.uniform(-1, 1, (300, dim)).astype(np.float32)
    q = rng.uniform(-1, 1, (3, dim)).astype(np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    ids = rng.permutation(300).astype(np.uint32)[:137]
    out = dev.distances(q, ids)
    for a in range(3):
        ref = np.array([orc.dist(metric, q[a], base[i]) for i in ids], np.float32)
        assert np.array_equal(out[a].view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("ef", [10, 20, 50, 100, 200])
def test_search_c1_bit_exact(native, orc, c1, ef):
    base, queries = c1
    g, view = _graph_view(native, orc, base)
    _check(view, _dev(native, base, g), queries, 10, ef)


@pytest.mark.parametrize("k,ef", [(1, 1), (1, 10), (10, 10), (3, 3), (16, 16), (100, 100), (64, 300)])
def test_search_k_ef_shapes(native, orc, c1, k, ef):
    base, queries = c1
    g, view = _graph_view(native, orc, base)
    _check(view, _dev(native, base, g), queries, k, ef)


@pytest.mark.parametrize("dim", [64, 128, 256])
@pytest.mark.parametrize("ef", [16, 64, 70, 127, 128, 129, 200])
def test_search_ties_pool_merge(native, orc, dim, ef):
    """Small-integer rows tie on most distances: the pool's (distance, arrival) order is all that
    separates them.  ef <= 128 runs the small-row kernels' register merge, ef > 128 the
    binary-search merge; both must match LinearPool::insert's order (the oracle)."""
    rng = np.random.default_rng(dim + ef)
    base = rng.integers(0, 3, (3000, dim)).astype(np.float32)
    queries = rng.integers(0, 3, (24, dim)).astype(np.float32)
    queries[:4] = base[:4]  # exact hits: distance 0 ties among duplicates
    g, view = _graph_view(native, orc, base)
    _check(view, _dev(native, base, g), queries, 10, ef)


def test_k_larger_than_ef(native, orc, c1):
    """k > ef reads past LinearPool's live entries in the reference (slot ef holds the last dropped
    neighbour, beyond it is out of bounds: query_utils.hpp:238, graph_search_job.hpp:254-256).
    The engine defines it: the first ef entries are the pool, the rest are (id 0, dist 0.0)."""
    base, queries = c1
    g, view = _graph_view(native, orc, base)
    ids, dists, _ = _dev(native, base, g).search(queries, 8, 5)
    for i, q in enumerate(queries):
        r_ids, r_d = view.search(q, 5, 5)
        assert np.array_equal(ids[i, :5], r_ids) and np.array_equal(dists[i, :5], r_d)
        assert not ids[i, 5:].any() and not dists[i, 5:].any()


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("log2", [6, 8, 11, 14])
def test_visited_spill_path(native, orc, c1, log2, mode):
    """Visited-table layouts (1 compact 16-bit, 2 wide 32-bit, 3 compact with probes capped at 2)
    at sizes from tiny (immediate spill to the per-slot global bitset) to roomy (no spill, and for
    C1's n=1000 ids narrower than the table); results must not change."""
    base, queries = c1
    g, view = _graph_view(native, orc, base)
    dev = _dev(native, base, g)
    dev.set_hash_log2(log2)
    dev.set_visited_mode(mode)
    _check(view, dev, queries, 10, 100)


@pytest.mark.parametrize("mode", [1, 3])
def test_visited_compact_wide_remainder(native, orc, mode):
    """Compact layout with many remainder bits (n = 70k ids, 2^6..2^9 slots: rbits 8..11, the
    largest encodable), so entries carry short probe distances; results must not change."""
    rng = np.random.default_rng(21)
    base = rng.random((70000, 16), dtype=np.float32)
    queries = rng.random((16, 16), dtype=np.float32)
    g, view = _graph_view(native, orc, base, threads=8)
    for log2 in (6, 9):
        dev = _dev(native, base, g)
        dev.set_hash_log2(log2)
        dev.set_visited_mode(mode)
        _check(view, dev, queries, 10, 200)


@pytest.mark.parametrize("metric", [1, 2])
def test_search_ip_cos(native, orc, metric):
    rng = np.random.default_rng(3 + metric)
    base = rng.standard_normal((2000, 96)).astype(np.float32)
    queries = rng.standard_normal((20, 96)).astype(np.float32)
    if metric == 2:
        base = np.stack([orc.normalize(r) for r in base])
        queries = np.stack([orc.normalize(r) for r in queries])
    g, view = _graph_view(native, orc, base, metric=metric)
    _check(view, _dev(native, base, g, metric), queries, 10, 64)


def test_search_gist_shaped(native, orc):
    rng = np.random.default_rng(9)
    centres = rng.uniform(0, 0.5, (16, 960)).astype(np.float32)
    base = np.clip(centres[rng.integers(0, 16, 6000)] + rng.normal(0, 0.05, (6000, 960)), 0, 1).astype(np.float32)
    queries = np.clip(centres[rng.integers(0, 16, 24)] + rng.normal(0, 0.05, (24, 960)), 0, 1).astype(np.float32)
    g, view = _graph_view(native, orc, base, threads=8)
    _check(view, _dev(native, base, g), queries, 10, 80)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("dim", [768, 960])
def test_two_waves_per_simd_wide_rows(native, orc, monkeypatch, dim, metric):
    """The wide-row f32 kernels at two waves per SIMD (one row per lane group, kMode 8), which a
    batch just past the one-wave kernel's resident searchers runs (config 4's S = 1 layout), forced
    here with ALAYA_TWO_WAVES=1: the same ids, distance bits and counters as the restatement."""
    monkeypatch.setenv("ALAYA_TWO_WAVES", "1")
    rng = np.random.default_rng(dim + metric)
    centres = rng.uniform(0, 0.5, (16, dim)).astype(np.float32)
    base = np.clip(centres[rng.integers(0, 16, 5000)] + rng.normal(0, 0.05, (5000, dim)), 0, 1).astype(np.float32)
    queries = np.clip(centres[rng.integers(0, 16, 40)] + rng.normal(0, 0.05, (40, dim)), 0, 1).astype(np.float32)
    g, view = _graph_view(native, orc, base, metric=metric, threads=8)
    _check(view, _dev(native, base, g, metric), queries, 10, 96)


def test_search_sift_shaped_many_queries(native, orc):
    rng = np.random.default_rng(4)
    base = rng.integers(0, 128, (20000, 128)).astype(np.float32)
    queries = rng.integers(0, 128, (3000, 128)).astype(np.float32)
    g, view = _graph_view(native, orc, base, threads=8)
    dev = _dev(native, base, g)
    ids, dists, cnt = dev.search(queries, 10, 40)
    sample = rng.choice(3000, 60, replace=False)
    for i in sample:
        r_ids, r_d = view.search(queries[i], 10, 40)
        assert np.array_equal(ids[i], r_ids) and np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32))


def test_invalid_rows_get_flt_max(native, orc, c1):
    """RawSpace::QueryComputer returns FLT_MAX for rows cleared in the validity bitmap
    (raw_space.hpp:298-300)."""
    base, queries = c1
    valid = np.full(1000 // 8, 0xFF, np.uint8)
    valid[3] = 0x5A
    valid[50] = 0x00
    g, view = _graph_view(native, orc, base, valid=valid)
    _check(view, _dev(native, base, g, valid=valid), queries, 10, 100)


def test_nsg_style_entry_points(native, orc, c1):
    base, queries = c1
    g0 = native.Graph.build(base, 0, 32, 100, 1, 100)
    l0 = g0.arrays()[0]
    eps = np.array([5, 77, 5, 901], np.uint32)  # repeated ep inserted twice, like the reference loop
    g = native.Graph.from_arrays(l0, None, None, None, 0, 0, eps)
    dev = _dev(native, base, g)
    ids, dists, cnt = dev.search(queries, 10, 50)
    for i, q in enumerate(queries):
        r_ids, r_d = _nsg_model(orc, base, l0, eps, q, 10, 50)
        assert np.array_equal(ids[i], r_ids) and np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32))


def _nsg_model(orc, base, l0, eps, q, k, ef):
    """Pure-Python restatement of search_solo with Graph::initialize_search's eps branch
    (graph.hpp:153-156), driving the oracle's LinearPool and distance."""
    pool = orc.Pool(base.shape[0], ef)
    vis = set()
    for e in eps:
        pool.insert(int(e), float(orc.l2(q, base[e])))
        vis.add(int(e))
    while pool.has_next():
        u = pool.pop()
        for v in l0[u]:
            if v == 0xFFFFFFFF:
                break
            if int(v) in vis:
                continue
            vis.add(int(v))
            pool.insert(int(v), float(orc.l2(q, base[v])))
    ids = np.array([pool.id(i) for i in range(k)], np.uint32)
    d = np.array([pool.dist(i) for i in range(k)], np.float32)
    return ids, d


def test_duplicate_edges_dedup(native, orc, c1):
    base, queries = c1
    g0 = native.Graph.build(base, 0, 32, 100, 1, 100)
    l0, levels, off, ue, ep, upper_r, _ = g0.arrays()
    l0 = l0.copy()
    for u in range(0, 1000, 3):  # repeat an earlier neighbour inside the row
        cnt = int((l0[u] != 0xFFFFFFFF).sum())
        if 2 <= cnt < 32:
            l0[u, cnt] = l0[u, 0]
    g = native.Graph.from_arrays(l0, levels, off, ue, upper_r, ep)
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep)
    _check(view, _dev(native, base, g), queries, 10, 50)


def test_index_api_end_to_end(native, orc, c1):
    import alayalite_amd

    base, queries = c1
    client = alayalite_amd.Client()
    index = client.create_index("c1", capacity=1000)
    index.fit(base, ef_construction=100, num_threads=1)
    ids = index.batch_search(queries, 10, 100)
    ids2, dists = index.batch_search_with_distance(queries, 10, 100)
    one = index.search(queries[0], 10, 100)
    assert ids.dtype == np.uint32 and ids.shape == (10, 10)
    assert np.array_equal(ids, ids2) and np.array_equal(one, ids[0])
    l0, levels, off, ue, ep, upper_r, _ = index.native().graph_arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep)
    for i, q in enumerate(queries):
        r_ids, r_d = view.search(q, 10, 100)
        assert np.array_equal(ids[i], r_ids) and np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32))
    from alayalite_amd.utils import calc_gt, calc_recall

    assert calc_recall(ids, calc_gt(base, queries, 10)) >= 0.9
    assert np.array_equal(index.get_data_by_id(7), base[7])


def test_index_save_load(native, c1, tmp_path):
    import alayalite_amd

    base, queries = c1
    client = alayalite_amd.Client(str(tmp_path))
    index = client.create_index("saved", capacity=2000)
    index.fit(base)
    before = index.batch_search(queries, 10, 50)
    client.save_index("saved")
    again = alayalite_amd.Client(str(tmp_path)).get_index("saved")
    assert np.array_equal(again.batch_search(queries, 10, 50), before)
    assert again.get_dim() == 128


def _typed_data(dtype, n, nq, d, seed):
    rng = np.random.default_rng(seed)
    if dtype == np.float64:
        return rng.standard_normal((n, d)), rng.standard_normal((nq, d))
    lo, hi = {np.int8: (-100, 100), np.uint8: (0, 256), np.int32: (-5000, 5000), np.uint32: (0, 9000)}[dtype]
    return rng.integers(lo, hi, (n, d)).astype(dtype), rng.integers(lo, hi, (nq, d)).astype(dtype)


@pytest.mark.parametrize("dtype", [np.int8, np.uint8, np.int32, np.uint32, np.float64])
@pytest.mark.parametrize("metric", ["l2", "ip"])
def test_non_float_dtypes_match_restatement(native, orc, dtype, metric):
    """A10: Index.fit / batch_search on int8, uint8, int32, uint32 and float64 rows.  The reference's
    RawSpace<T> compares them with the generic branch of l2_sqr<T>/ip_sqr<T> (distance_l2.ipp:735-741,
    distance_ip.ipp:744-750): elements cast to float, summed into one float accumulator.  Graph =
    the oracle's builder (generic order); search ids and distance bits = the oracle's search.

    What this pins: for int8 / uint8 rows (d = 24) every partial sum is an integer below 2^24, so
    any summation order gives the same float -- equality with the restatement is equality with the
    reference.  For int32 / uint32 / float64 the partial sums are not exact in float and the order
    is visible; the reference is built with -Ofast (CMakeLists.txt:34), which lets GCC vectorise the
    loop into strided partial sums.  There the test compares against the restatement's in-order sum
    only: parity with the reference binary is unpinned."""
    import alayalite_amd

    base, queries = _typed_data(dtype, 2500, 24, 48, 70 + (metric == "ip"))
    index = alayalite_amd.Client().create_index(f"t_{np.dtype(dtype).name}_{metric}", capacity=2500, data_type=dtype,
                                                metric=metric)
    index.fit(base, ef_construction=100, num_threads=1)
    ids, dists = index.batch_search_with_distance(queries, 10, 64)
    l0, levels, off, ue, ep, upper_r, _ = index.native().graph_arrays()
    rows, qf = base.astype(np.float32), queries.astype(np.float32)
    m = 0 if metric == "l2" else 1
    o_l0, o_levels, o_off, o_ue, o_ep, _ = orc.build_hnsw(rows, m, 32, 100, 100, generic=True)
    assert np.array_equal(l0, o_l0) and np.array_equal(ue, o_ue) and ep == o_ep
    view = orc.IndexView(rows, l0, levels, off, ue, upper_r, ep, metric=m, generic=True)
    for i in range(len(qf)):
        r_ids, r_d = view.search(qf[i], 10, 64)
        assert np.array_equal(ids[i].astype(np.uint32), r_ids), i
        assert np.array_equal(dists[i].view(np.uint32), r_d.view(np.uint32)), i


def test_uint64_ids_and_int_dtype(native, c1):
    import alayalite_amd

    rng = np.random.default_rng(1)
    base = rng.integers(0, 50, (1000, 64)).astype(np.int32)
    queries = rng.integers(0, 50, (5, 64)).astype(np.int32)
    index = alayalite_amd.Client().create_index("u64", capacity=1000, id_type=np.uint64, data_type=np.int32)
    index.fit(base)
    ids = index.batch_search(queries, 10, 100)
    assert ids.dtype == np.uint64
    from alayalite_amd.utils import calc_gt, calc_recall

    assert calc_recall(ids, calc_gt(base, queries, 10)) >= 0.9

