"""Online updates: Index.insert / Index.remove.

Reference: PyIndex::insert/remove (python/include/index.hpp:229-234) -> GraphUpdateJob
insert_and_update / update / remove (include/executor/jobs/graph_update_job.hpp:49-137), JobContext
(job_context.hpp:25-29).  CPU: the restatement (oracle.Updater) against the reference's own update
test (tests/executor/update_test.cpp HalfInsertTest: recall > 0.9 after inserting the second half).
GPU: the engine's adjacency rows and search results after mixed insert/remove sequences are
bit-identical to the restatement's; python/tests/test_update.py's API cases.
"""

import numpy as np
import pytest


def _exact_l2(base, q, k, exclude=()):
    d = ((base[None, :, :] - q[:, None, :]) ** 2).sum(-1)
    if exclude:
        d[:, list(exclude)] = np.inf
    return np.argsort(d, axis=1, kind="stable")[:, :k]


def _recall(ids, gt):
    return np.mean([len(set(a.tolist()) & set(b.tolist())) / len(b) for a, b in zip(ids, gt)])


def test_restated_half_insert_recall(native, orc):
    """update_test.cpp HalfInsertTest on a SIFT-small-shaped sample: build on the first half,
    insert_and_update the second half at ef=50, recall@10 at ef=50 stays > 0.9."""
    rng = np.random.default_rng(21)
    centres = rng.uniform(0, 64, (40, 32)).astype(np.float32)
    data = (centres[rng.integers(0, 40, 2000)] + rng.normal(0, 6, (2000, 32))).astype(np.float32)
    queries = (centres[rng.integers(0, 40, 50)] + rng.normal(0, 6, (50, 32))).astype(np.float32)
    half = 1000
    g = native.Graph.build(data[:half], 0, 32, 100, 1, 100)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    view = orc.IndexView(data[:half], l0, levels, off, ue, ur, ep)
    up = orc.Updater(view, 2000)
    for i in range(half, 2000):
        assert up.insert(data[i], data[i], 50) == i
    assert up.n() == 2000
    ids = np.stack([up.search(q, 10, 50)[0] for q in queries])
    assert _recall(ids, _exact_l2(data, queries, 10)) > 0.9
    # removed rows score FLT_MAX: with a full pool they never reach the top-10
    removed = list(range(half, half + 300))
    for r in removed:
        up.remove(r)
    ids = np.stack([up.search(q, 10, 100)[0] for q in queries])
    assert not set(ids.ravel().tolist()) & set(removed)


def test_restated_update_pads_with_zero(native, orc):
    """update() copies pool ids into a value-initialised vector: a node with fewer than R
    candidates gets 0 (not -1) in its trailing slots (graph_update_job.hpp:131-135)."""
    rng = np.random.default_rng(3)
    data = rng.random((6, 8), dtype=np.float32)
    g = native.Graph.build(data[:5], 0, 32, 100, 1, 100)
    l0, levels, off, ue, ep, ur, _ = g.arrays()
    up = orc.Updater(orc.IndexView(data[:5], l0, levels, off, ue, ur, ep), 6)
    assert up.insert(data[5], data[5], 40) == 5
    rows = up.l0()
    # every pre-existing node gained the new node; its row is now pool ids then zeros
    for u in range(5):
        row = rows[u]
        assert 5 in row.tolist()
        assert (row[5:] == 0).all() and 0xFFFFFFFF not in row.tolist()
    assert up.insert(data[0], data[0], 40) == -1  # capacity reached


def _engine_vs_restatement(native, orc, metric, seed, client=None):
    import alayalite_amd

    rng = np.random.default_rng(seed)
    n0, d = 600, 24
    base = rng.standard_normal((n0 + 200, d)).astype(np.float32)
    mname = {0: "l2", 1: "ip", 2: "cosine"}[metric]
    client = client or alayalite_amd.Client()
    idx = client.create_index(f"upd{metric}_{seed}", metric=mname, capacity=n0 + 150)
    fit_rows = base[:n0].copy()
    idx.fit(fit_rows, ef_construction=100, num_threads=1)  # COS normalises fit_rows in place
    l0, levels, off, ue, ep, ur, _ = idx._Index__index.graph_arrays()
    view = orc.IndexView(fit_rows, l0, levels, off, ue, ur, ep, metric=metric)
    up = orc.Updater(view, n0 + 150)
    ops = []
    for i in range(n0, n0 + 120):
        ops.append(("ins", i))
        if i % 7 == 0:
            ops.append(("rm", int(rng.integers(0, i))))
    for op, arg in ops:
        if op == "ins":
            v = base[arg].copy()
            if metric == 2:
                q1 = orc.normalize(v)
                row = orc.normalize(q1)
            else:
                q1 = row = v
            want = up.insert(q1, row, 48)
            got = idx.insert(base[arg].copy(), 48)
            assert got == want
        else:
            up.remove(arg)
            idx.remove(arg)
    l0_dev, *_ = idx._Index__index.graph_arrays()
    assert np.array_equal(l0_dev, up.l0())
    qs = rng.standard_normal((16, d)).astype(np.float32)
    for q in qs:
        qq = orc.normalize(q) if metric == 2 else q
        ids, dists = idx.batch_search_with_distance(q.reshape(1, -1).copy(), 10, 64)
        o_ids, o_d = up.search(qq, 10, 64)
        assert np.array_equal(ids[0].astype(np.uint32), o_ids)
        assert np.array_equal(dists[0].view(np.uint32), o_d.view(np.uint32))
    return idx, up


@pytest.mark.gpu
@pytest.mark.parametrize("metric", [0, 1, 2])
def test_insert_remove_bit_exact(native, orc, metric):
    _engine_vs_restatement(native, orc, metric, 40 + metric)


@pytest.mark.gpu
def test_insert_api_like_reference():
    """python/tests/test_update.py: ids 1000, 1001, get_data_by_id, RuntimeError when full."""
    import alayalite_amd

    client = alayalite_amd.Client()
    index = client.create_index("upd_api")
    vectors = np.random.default_rng(0).random((1000, 128), dtype=np.float32)
    index.fit(vectors)
    v1 = np.random.default_rng(1).random(128, dtype=np.float32)
    v2 = np.random.default_rng(2).random(128, dtype=np.float32)
    assert index.insert(v1) == 1000
    assert index.insert(v2) == 1001
    assert np.allclose(index.get_data_by_id(1000), v1)
    assert np.allclose(index.get_data_by_id(1001), v2)
    # the inserted vector is found by search
    assert index.batch_search(v1.reshape(1, -1).copy(), 1, 100)[0, 0] == 1000
    full = client.create_index("upd_full", capacity=1000)
    full.fit(vectors)
    with pytest.raises(RuntimeError):
        full.insert(v1)


@pytest.mark.gpu
def test_updates_survive_save_load(native, orc, tmp_path):
    import alayalite_amd

    client = alayalite_amd.Client(str(tmp_path))
    idx, up = _engine_vs_restatement(native, orc, 0, 77, client)
    client.save_index("upd0_77")
    again = alayalite_amd.Client(str(tmp_path)).get_index("upd0_77")
    l0, *_ = again._Index__index.graph_arrays()
    assert np.array_equal(l0, up.l0())
    q = np.random.default_rng(5).standard_normal((4, 24)).astype(np.float32)
    assert np.array_equal(again.batch_search(q.copy(), 10, 64), idx.batch_search(q.copy(), 10, 64))
