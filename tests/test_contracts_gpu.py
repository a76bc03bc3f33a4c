"""Boundary contracts of the device index (the C ABI, include/alaya_hip.h) that round 1's advisor
review flagged: validity-bitmap handling on the flat path, the graph file's storage bitmap after
remove(), SQ8 codes invalidated by a new base, and calls on one index from two HIP streams."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _exact_valid(orc, base, q, k, valid_rows):
    out = []
    for a in range(len(q)):
        d = np.array([orc.l2(q[a], base[i]) for i in range(len(base))], np.float32)
        d[~valid_rows] = np.inf
        o = np.lexsort((np.arange(len(base)), d))[:k]
        out.append((o.astype(np.uint32), d[o]))
    return out


@pytest.mark.parametrize("d,k", [(64, 10), (960, 10), (64, 50)])
@pytest.mark.parametrize("f32", [False, True])
def test_flat_skips_invalid_rows(native, orc, monkeypatch, f32, d, k):
    """Rows cleared in the validity bitmap (removed rows) are never returned by the flat path, on
    the MFMA shortlist path and on the exhaustive recompute of a flagged query alike."""
    monkeypatch.delenv("ALAYA_FLAT_PRESCAN", raising=False)
    if f32:
        monkeypatch.setenv("ALAYA_FLAT_F32", "1")
    else:
        monkeypatch.delenv("ALAYA_FLAT_F32", raising=False)
    rng = np.random.default_rng(31)
    n = 3000  # d = 64: the warp-specialised (split) or single-role (f32) scan; 960: the slabbed scan
    base = rng.random((n, d), dtype=np.float32)
    q = rng.random((12, d), dtype=np.float32)
    # invalidate each query's 5 nearest rows plus a block of rows
    valid_rows = np.ones(n, bool)
    for a in range(len(q)):
        dd = ((base - q[a]) ** 2).sum(1)
        valid_rows[np.argsort(dd)[:5]] = False
    valid_rows[100:164] = False
    bitmap = np.packbits(valid_rows.astype(np.uint8), bitorder="little")
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0, bitmap)
    ids, dists, _ = dev.flat_search(q, k)
    for a, (ri, rd) in enumerate(_exact_valid(orc, base, q, k, valid_rows)):
        assert np.array_equal(ids[a], ri), a
        assert np.array_equal(dists[a].view(np.uint32), rd.view(np.uint32)), a
    # all-tied rows force the exhaustive recompute: still only valid rows
    tied = np.tile(rng.random(d, dtype=np.float32), (400, 1))
    v2 = np.ones(400, bool)
    v2[::2] = False
    dev.set_base(tied, 0, np.packbits(v2.astype(np.uint8), bitorder="little"))
    ids, _, redo = dev.flat_search(q[:2], 10)
    assert redo == 2
    assert (ids == np.arange(1, 21, 2, dtype=np.uint32)).all()


def test_flat_fewer_rows_than_k(native):
    """n < k: the result holds every row, then empty slots (0xffffffff, FLT_MAX)."""
    rng = np.random.default_rng(4)
    base = rng.random((6, 32), dtype=np.float32)
    q = rng.random((3, 32), dtype=np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, _ = dev.flat_search(q, 10)
    for a in range(3):
        assert sorted(ids[a, :6].tolist()) == list(range(6))
        assert (ids[a, 6:] == 0xFFFFFFFF).all() and (dists[a, 6:] == np.finfo(np.float32).max).all()


def test_saved_graph_bitmap_records_removals(native, tmp_path):
    """Graph::remove clears the node's storage bit (sequential_storage.hpp:94-100), so the
    reference's .index file records the removal; the engine's file does the same."""
    import alayalite_amd

    rng = np.random.default_rng(8)
    base = rng.random((300, 16), dtype=np.float32)
    client = alayalite_amd.Client(str(tmp_path))
    idx = client.create_index("rm", capacity=400)
    idx.fit(base)
    for r in (3, 17, 299):
        idx.remove(r)
    client.save_index("rm")
    path = tmp_path / "rm" / "hnsw_l2_32.index"
    raw = path.read_bytes()
    # header: int32 nep (0), u32 max_nodes, u32 max_nbrs, then 5 x u64 storage header
    item, aligned, cap, pos = np.frombuffer(raw, np.uint64, 4, 12)
    assert (cap, pos) == (400, 300)
    bitmap = np.frombuffer(raw, np.uint8, (int(cap) + 7) // 8, 12 + 40 + int(aligned) * int(cap))
    bits = np.unpackbits(bitmap, bitorder="little")[:400].astype(bool)
    want = np.zeros(400, bool)
    want[:300] = True
    want[[3, 17, 299]] = False
    assert np.array_equal(bits, want)


def test_new_base_invalidates_sq8_codes(native):
    rng = np.random.default_rng(5)
    base = rng.random((500, 32), dtype=np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    g, _ = dev.build_graph(32, 100, 100, 0, 0, 2)
    mn, mx = native.sq8_train(base)
    dev.set_sq8(native.sq8_encode(base, mn, mx, 4), mn, mx, 2)
    dev.search_sq8(base[:2], 10, 20, 0, None)
    bigger = rng.random((900, 32), dtype=np.float32)
    dev.set_base(bigger, 0)
    dev.set_graph(native.Graph.build(bigger, 0, 32, 100, 4, 100))
    with pytest.raises(ValueError, match="no SQ8 codes"):
        dev.search_sq8(bigger[:2], 10, 20, 0, None)


def test_same_shape_base_invalidates_sq8_codes(native):
    """A replacement base of the same shape must drop the codes too: they describe the old rows."""
    rng = np.random.default_rng(6)
    base = rng.random((500, 32), dtype=np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(native.Graph.build(base, 0, 32, 100, 4, 100))
    mn, mx = native.sq8_train(base)
    dev.set_sq8(native.sq8_encode(base, mn, mx, 4), mn, mx, 2)
    dev.search_sq8(base[:2], 10, 20, 0, None)
    other = rng.random((500, 32), dtype=np.float32)
    dev.set_base(other, 0)
    with pytest.raises(ValueError, match="no SQ8 codes"):
        dev.search_sq8(other[:2], 10, 20, 0, None)


def test_two_streams_one_index(native, orc):
    """Launches on two HIP streams share the index's scratch (work counter, spill area); the
    engine orders the second call after the first, so both batches come out exact."""
    import torch

    rng = np.random.default_rng(12)
    base = rng.random((20000, 64), dtype=np.float32)
    qa = rng.random((2000, 64), dtype=np.float32)
    qb = rng.random((2000, 64), dtype=np.float32)
    g = native.Graph.build(base, 0, 32, 100, 8, 100)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    dev.set_graph(g)
    d0 = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(d0), torch.cuda.Stream(d0)
    outs = []
    for q, s in ((qa, s1), (qb, s2)):
        qd = torch.from_numpy(q).to(d0)
        torch.cuda.synchronize()
        ids = torch.empty((len(q), 10), dtype=torch.int32, device=d0)
        dd = torch.empty((len(q), 10), dtype=torch.float32, device=d0)
        cc = torch.empty((len(q), 4), dtype=torch.int32, device=d0)
        dev.search_device(qd.data_ptr(), len(q), 10, 200, ids.data_ptr(), dd.data_ptr(), cc.data_ptr(),
                          s.cuda_stream)
        outs.append((q, qd, ids, dd))
    torch.cuda.synchronize()
    l0, levels, off, ue, ep, upper_r, _ = g.arrays()
    view = orc.IndexView(base, l0, levels, off, ue, upper_r, ep)
    for q, _, ids, dd in outs:
        got = ids.cpu().numpy().astype(np.uint32)
        for i in range(0, len(q), 97):
            r_ids, r_d = view.search(q[i], 10, 200)
            assert np.array_equal(got[i], r_ids), i
