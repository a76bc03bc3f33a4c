"""SQ8 search space (SQ8Space, space/sq8_space.hpp) and PyIndex::rerank (index.hpp:450-488).

CPU: the engine's quantizer equals the restatement's bit for bit; the rerank restatement shows the
reference's id-0 quirk.  GPU: SQ8 graph search (AVX-512 and AVX2 reduction orders) and the rerank
are bit-exact against the restatement; the Index API reproduces batch_search / _with_distance."""

import numpy as np
import pytest


def _data(n, d, nq, seed):
    rng = np.random.default_rng(seed)
    base = rng.standard_normal((n, d)).astype(np.float32)
    q = rng.standard_normal((nq, d)).astype(np.float32)
    return base, q


def test_quantizer_matches_restatement(native, orc):
    base, q = _data(500, 100, 5, 1)
    mn, mx = native.sq8_train(base)
    omn, omx = orc.sq8_fit(base)
    assert np.array_equal(mn, omn) and np.array_equal(mx, omx)
    codes = native.sq8_encode(base, mn, mx, 4)
    assert np.array_equal(codes, orc.sq8_encode(base, omn, omx))
    # queries outside the trained range clamp to 0 / 255
    qc = native.sq8_encode(q * 10, mn, mx, 1)
    assert np.array_equal(qc, orc.sq8_encode(q * 10, omn, omx))
    assert qc.min() == 0 and qc.max() == 255


def test_rerank_restatement_repeats_id0(native, orc):
    """batch_search writes k ids into a zero-filled ef-sized res_pool; rerank rescoring all ef
    entries makes id 0 appear ef-k times when row 0 is close to the query."""
    base, _ = _data(300, 32, 1, 2)
    g = native.Graph.build(base, 0, 32, 100, 1, 100)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, ur, ep)
    q = base[0] + 0.01
    ids, d = view.rerank(q, np.array([5, 6, 7], np.uint32), 3, 8)
    assert ids.tolist() == [0, 0, 0]  # five zeros in res_pool, row 0 is the nearest
    ids, d = view.rerank(q, np.array([0, 6, 7], np.uint32), 3, 3)
    assert ids[0] == 0 and len(set(ids.tolist())) == 3


def _sq8_setup(native, orc, n, d, nq, metric, seed, order):
    base, q = _data(n, d, nq, seed)
    if metric == 2:
        base = np.stack([orc.normalize(r) for r in base])
    g = native.Graph.build(base, metric, 32, 100, 4, 100)
    mn, mx = native.sq8_train(base)
    codes = native.sq8_encode(base, mn, mx, 4)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, ur, ep, metric=metric, sq8=(codes, mn, mx, order))
    return base, q, g, codes, mn, mx, view


@pytest.mark.gpu
@pytest.mark.parametrize("order", [2, 1])
@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("d", [128, 768, 960, 100, 48, 40, 24, 7])
def test_sq8_search_and_rerank_bit_exact(native, orc, order, metric, d):
    base, q, g, codes, mn, mx, view = _sq8_setup(native, orc, 1500, d, 12, metric, d + order, order)
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, order)
    k, ef = 10, 40
    s_ids, s_d, s_c = dev.search_sq8(q, k, ef, False)
    r_ids, r_d, _ = dev.search_sq8(q, k, ef, True)
    for i in range(len(q)):
        o_ids, o_d, o_c = view.search(q[i], k, ef, with_counters=True)
        assert np.array_equal(s_ids[i], o_ids), (i, s_ids[i], o_ids)
        assert np.array_equal(s_d[i].view(np.uint32), o_d.view(np.uint32))
        assert tuple(s_c[i]) == tuple(o_c)
        rr_ids, rr_d = view.rerank(q[i], o_ids, k, ef)
        assert np.array_equal(r_ids[i], rr_ids), (i, r_ids[i], rr_ids)
        assert np.array_equal(r_d[i].view(np.uint32), rr_d.view(np.uint32))


@pytest.mark.gpu
def test_sq8_rerank_quirk_on_device(native, orc):
    base, q, g, codes, mn, mx, view = _sq8_setup(native, orc, 400, 32, 1, 0, 3, 2)
    q = (base[0] + 0.001).reshape(1, -1).astype(np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    ids, d, _ = dev.search_sq8(q, 5, 50, True)
    o_ids, _ = view.search(q[0], 5, 50)
    rr_ids, rr_d = view.rerank(q[0], o_ids, 5, 50)
    assert np.array_equal(ids[0], rr_ids) and rr_ids[0] == 0 and (rr_ids == 0).sum() >= 2


@pytest.mark.gpu
@pytest.mark.parametrize("metric", [0, 1])
def test_sq8_corrected_rerank(native, orc, metric):
    """rerank=2 (SURVEY A12 corrected mode): the whole ef pool of the SQ8 search is rescored with
    the exact f32 metric and the k smallest (dist, id) come back -- no id-0 padding entries."""
    base, q, g, codes, mn, mx, view = _sq8_setup(native, orc, 1200, 64, 8, metric, 11 + metric, 2)
    dev = native.DeviceIndex(0)
    dev.set_base(base, metric)
    dev.set_graph(g)
    dev.set_sq8(codes, mn, mx, 2)
    k, ef = 10, 48
    ids, d, _ = dev.search_sq8(q, k, ef, 2)
    for i in range(len(q)):
        pool_ids, _ = view.search(q[i], ef, ef)  # the search's whole pool, in pool order
        ex = np.array([orc.dist(metric, q[i], base[j]) for j in pool_ids], np.float32)
        order = sorted(range(ef), key=lambda j: (ex[j], pool_ids[j]))[:k]
        assert np.array_equal(ids[i], pool_ids[order]), (i, ids[i], pool_ids[order])
        assert np.array_equal(d[i].view(np.uint32), ex[order].view(np.uint32))
        assert len(set(ids[i].tolist())) == k
    # a pool shorter than ef (tiny graph): slots past the candidates are (0, 0.0)
    small = base[:20].copy()
    gs = native.Graph.build(small, metric, 32, 100, 1, 100)
    mn2, mx2 = native.sq8_train(small)
    dev2 = native.DeviceIndex(0)
    dev2.set_base(small, metric)
    dev2.set_graph(gs)
    dev2.set_sq8(native.sq8_encode(small, mn2, mx2, 1), mn2, mx2, 2)
    ids2, d2, _ = dev2.search_sq8(q[:1], 25, 40, 2)
    assert sorted(ids2[0][:20].tolist()) == list(range(20))
    assert ids2[0][20:].tolist() == [0] * 5 and d2[0][20:].tolist() == [0.0] * 5


@pytest.mark.gpu
@pytest.mark.parametrize("metric", ["l2", "ip", "cosine"])
def test_sq8_index_api(native, orc, metric, tmp_path):
    import alayalite_amd

    rng = np.random.default_rng(7)
    base = rng.standard_normal((2000, 64)).astype(np.float32)
    queries = rng.standard_normal((16, 64)).astype(np.float32)
    client = alayalite_amd.Client(str(tmp_path))
    index = client.create_index("sq", capacity=2000, quantization_type="sq8", metric=metric)
    index.fit(base.copy())
    ids = index.batch_search(queries.copy(), 10, 60)
    ids2, dists = index.batch_search_with_distance(queries.copy(), 10, 60)
    assert dists.shape == (0, 10)  # reference: no distances for SQ spaces
    m = {"l2": 0, "ip": 1, "cosine": 2}[metric]
    fb = np.stack([orc.normalize(r) for r in base]) if m == 2 else base
    fq = np.stack([orc.normalize(r) for r in queries]) if m == 2 else queries
    l0, levels, off, ue, ep, ur, _ = index.native().graph_arrays()
    mn, mx = orc.sq8_fit(fb)
    codes = orc.sq8_encode(fb, mn, mx)
    order = native.host_sq8_order()
    view = orc.IndexView(fb, l0, levels, off, ue, ur, ep, metric=m, sq8=(codes, mn, mx, order))
    for i in range(len(queries)):
        o_ids, _ = view.search(queries[i], 10, 60)  # SQ8 search encodes the un-normalised query
        assert np.array_equal(ids2[i], o_ids)
        rr_ids, _ = view.rerank(fq[i], o_ids, 10, 60)
        assert np.array_equal(ids[i], rr_ids)
    client.save_index("sq")
    again = alayalite_amd.Client(str(tmp_path)).get_index("sq")
    assert np.array_equal(again.batch_search(queries.copy(), 10, 60), ids)
