"""Flat exact k-NN (BASELINE config 2's path; no reference implementation -- IndexType::FLAT is
enum-only).  Contract: the k smallest rows by the reference metric function (the l2_sqr_avx2-order
device distance, bit-identical to the CPU restatement) with ties broken by id."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["f16", "split", "f32", "f16-prescan2", "f32-prescan3", "f16-ws", "f16-ws1", "split-ws1"],
                autouse=True)
def flat_mode(request, monkeypatch):
    """Every shortlist contraction: the single-pass f16 on power-of-two-scaled operands (the default
    for rows of <= 224 floats), the bf16 hi/lo split (ALAYA_FLAT_CONTRACTION=bf16x3; the default for
    wider rows) and the f32 MFMA (ALAYA_FLAT_CONTRACTION=f32).  The exact rescoring and the bound
    check make the answer identical.  The single pass runs the single-role scan over the index's
    cached f16 tile records by default; -ws modes force the warp-specialised scan
    (ALAYA_FLAT_TILES=0), which converts the f32 rows itself.  The prescan (a scan over every S-th
    row -- every S-th tile record in the single-role scan -- that seeds each chunk's threshold;
    ALAYA_FLAT_PRESCAN=S) is forced on by the -prescanS modes.  The warp-specialised scan runs two
    consumer waves per producer by default; -ws1 forces one (ALAYA_FLAT_WS2=0)."""
    for var in ("ALAYA_FLAT_F32", "ALAYA_FLAT_PRESCAN", "ALAYA_FLAT_WS2", "ALAYA_FLAT_CONTRACTION",
                "ALAYA_FLAT_TILES"):
        monkeypatch.delenv(var, raising=False)
    if "-ws" in request.param:
        monkeypatch.setenv("ALAYA_FLAT_TILES", "0")
    if request.param.endswith("-ws1"):
        monkeypatch.setenv("ALAYA_FLAT_WS2", "0")
    if request.param.startswith("f32"):
        monkeypatch.setenv("ALAYA_FLAT_CONTRACTION", "f32")
    if request.param.startswith("split"):
        monkeypatch.setenv("ALAYA_FLAT_CONTRACTION", "bf16x3")
    if "prescan" in request.param:
        monkeypatch.setenv("ALAYA_FLAT_PRESCAN", request.param[-1])
    return request.param


def _contraction_of(mode, dim):
    """The contraction a flat search in this mode runs (alaya_index_flat_last_contraction)."""
    if mode.startswith("f32"):
        return 0
    if mode.startswith("split") or (dim + 31) // 32 * 32 > 224:
        return 1
    return 2


def _exact(orc, base, q, k):
    lib = orc.lib()
    out_i = np.zeros((len(q), k), np.uint32)
    out_d = np.zeros((len(q), k), np.float32)
    for a in range(len(q)):
        qa = np.ascontiguousarray(q[a])
        d = np.array([lib.orc_l2_f32(orc._ptr(qa), orc._ptr(base[i]), base.shape[1]) for i in range(len(base))],
                     np.float32)
        o = np.lexsort((np.arange(len(base)), d))[:k]
        out_i[a], out_d[a] = o, d[o]
    return out_i, out_d


@pytest.mark.parametrize("n,d,nq", [(5000, 128, 37), (3000, 32, 130), (2500, 100, 9), (4000, 200, 64),
                                    (2000, 224, 5), (777, 64, 300),
                                    # the remaining narrow strides (96, 160, 192 floats): every
                                    # instantiation of the single-role and warp-specialised scans
                                    (3000, 96, 33), (2600, 150, 21), (2400, 180, 70)])
def test_flat_exact(native, orc, flat_mode, n, d, nq):
    rng = np.random.default_rng(n + d)
    base = np.ascontiguousarray(rng.random((n, d), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((nq, d), dtype=np.float32))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    assert dev.flat_contraction() == _contraction_of(flat_mode, d)
    ref_i, ref_d = _exact(orc, base, q, 10)
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))
    assert redo == 0  # the shortlist bound is proven on every query of continuous data


@pytest.mark.parametrize("scale,shift", [(1e3, 0.0), (1e-3, 0.0), (1.0, -0.5), (1e-20, 1e-21)])
def test_flat_exact_scaled(native, orc, scale, shift):
    """Signed, large and tiny magnitudes: the f16 operands are scaled by powers of two into range
    (at 1e-20 the row scale 2^s leaves the f16 pass's range and the split runs, with bf16 lo parts in
    the denormal range); each contraction's error bound scales with |q||b|, so the answer stays
    exact."""
    rng = np.random.default_rng(7)
    base = np.ascontiguousarray((rng.standard_normal((3000, 96)) * scale + shift).astype(np.float32))
    q = np.ascontiguousarray((rng.standard_normal((40, 96)) * scale + shift).astype(np.float32))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    ref_i, ref_d = _exact(orc, base, q, 10)
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))


@pytest.mark.parametrize("n,d,nq,k", [(3000, 256, 20, 10), (2500, 300, 17, 10), (3000, 768, 12, 10),
                                      (4000, 960, 10, 10), (2000, 960, 150, 24), (1500, 1000, 6, 5)])
def test_flat_exact_wide_rows(native, orc, n, d, nq, k):
    """Rows wider than the narrow scan's 224 floats: the slabbed scan (K cut into slabs, TT row
    tiles per super-chunk, zero-padded queries) feeds the same shortlists and exact rescoring."""
    rng = np.random.default_rng(n + d + k)
    base = np.ascontiguousarray(rng.random((n, d), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((nq, d), dtype=np.float32))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, k)
    ref_i, ref_d = _exact(orc, base, q, k)
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))
    if k <= 10:
        # uniform 960-d distances concentrate: with k = 24 the gap to the 32nd shortlist entry can
        # fall inside the split contraction's error bound, and those queries are recomputed
        assert redo == 0


@pytest.mark.parametrize("n,d,nq,k", [(6000, 128, 20, 50), (6000, 128, 9, 100), (5000, 64, 7, 224),
                                      (4000, 960, 8, 100), (3000, 200, 5, 25)])
def test_flat_exact_large_k(native, orc, n, d, nq, k):
    """k past the 32-entry chunk shortlists: the merge folds them into a 128- or 256-entry
    register list and proves the k-th result against min(list end, every chunk's 32nd)."""
    rng = np.random.default_rng(3 * n + d + k)
    base = np.ascontiguousarray(rng.random((n, d), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((nq, d), dtype=np.float32))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, k)
    ref_i, ref_d = _exact(orc, base, q, k)
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))


def test_flat_f16_query_scale_out_of_range(native, orc, flat_mode):
    """Queries whose own f16 scale-back 2^-(s+t) would leave f32's range (1e-30-sized queries against
    rows of norm ~6): with per-query scales (the warp-specialised scan) the merge flags them and more
    than 1 % flagged reruns the launch with the split; with the single-role scan's per-wave scale
    they are proven as they are.  The answer is exact either way."""
    rng = np.random.default_rng(17)
    base = np.ascontiguousarray(rng.random((4000, 64), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((20, 64), dtype=np.float32))
    q[::4] *= np.float32(1e-30)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    ref_i, ref_d = _exact(orc, base, q, 10)
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))
    if flat_mode == "f16-ws":  # per-query scales: five of twenty flagged, the launch reran with the split
        assert dev.flat_contraction() == 1
    # the single-role scan scales each wave of 32 queries by its largest element, so the tiny
    # queries' operands flush to zero and the bound's absolute term (2^-14-t |b|) proves them


def test_flat_rejects_unsupported(native):
    dev = native.DeviceIndex(0)
    dev.set_base(np.zeros((100, 300), np.float32), 0)
    with pytest.raises(ValueError, match="k <= 224"):
        dev.flat_search(np.zeros((1, 300), np.float32), 225)


def test_flat_ties_and_fallback(native, orc):
    """Identical rows: every distance ties, so the shortlist bound cannot be proven -- the host
    recomputes exhaustively and the answer is ids 0..k-1 (ties by id)."""
    rng = np.random.default_rng(1)
    row = rng.random(64, dtype=np.float32)
    base = np.tile(row, (600, 1))
    q = rng.random((3, 64), dtype=np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    assert redo == 3
    assert (ids == np.arange(10, dtype=np.uint32)).all()


def test_flat_spin_abort_is_flagged_and_redone(native, orc, flat_mode, monkeypatch):
    """The warp-specialised scan gives up on an LDS flag after ALAYA_FLAT_SPIN_LIMIT polls: its
    consumers then write unprovable shortlists.  Forced with a zero limit, the device entry flags
    every query of an aborted consumer (aligned blocks of 16 queries with two consumers per producer,
    32 with one, all or none), and flat_search's
    exhaustive redo still returns the exact answer."""
    import torch

    if flat_mode not in ("f16-ws", "f16-ws1", "split", "split-ws1"):
        pytest.skip("the ring protocol belongs to the warp-specialised scan (f16 and split contractions)")
    group = 32 if flat_mode.endswith("-ws1") else 16  # queries per consumer wave
    monkeypatch.setenv("ALAYA_FLAT_SPIN_LIMIT", "0")
    rng = np.random.default_rng(44)
    base = np.ascontiguousarray(rng.random((20000, 128), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((256, 128), dtype=np.float32))
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    d0 = torch.device("cuda", 0)
    qd = torch.from_numpy(q).to(d0)
    ids_d = torch.empty((256, 10), dtype=torch.int32, device=d0)
    dd = torch.empty((256, 10), dtype=torch.float32, device=d0)
    flags = torch.zeros((256,), dtype=torch.int32, device=d0)
    s = torch.cuda.current_stream(d0)
    dev.flat_search_device(qd.data_ptr(), 256, 10, ids_d.data_ptr(), dd.data_ptr(), flags.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    f = flags.cpu().numpy().reshape(-1, group)
    assert f.sum() > 0  # 20k rows of 32-row tiles: a zero poll limit trips on some hand-over
    assert ((f == 0).all(1) | (f != 0).all(1)).all()
    ids, dists, redo = dev.flat_search(q[:16], 10)
    ref_i, ref_d = _exact(orc, base, q[:16], 10)
    assert redo > 0
    assert np.array_equal(ids, ref_i)
    assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))


def test_flat_duplicates_sift_like(native, orc):
    rng = np.random.default_rng(2)
    base = rng.integers(0, 4, (3000, 32)).astype(np.float32)  # many exact ties
    q = rng.integers(0, 4, (20, 32)).astype(np.float32)
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    ref_i, ref_d = _exact(orc, base, q, 10)
    assert np.array_equal(ids, ref_i) and np.array_equal(dists, ref_d)


@pytest.fixture(scope="module")
def flat_1m(orc):
    """Config 2 at full size: 1M x 128 rows and 1,000 queries -- the bench's launch shape (8 query
    groups of 128 per chunk, the last one partial); the oracle's find_exact_gt restatement on 16
    threads (continuous data: no ties to order)."""
    rng = np.random.default_rng(1_000_000)
    base = rng.random((1_000_000, 128), dtype=np.float32)
    q = rng.random((1000, 128), dtype=np.float32)
    ref_i, _ = orc.exact_gt(base, q, 10, num_threads=16)
    return base, q, ref_i.astype(np.uint32)


def test_flat_exact_1m(native, orc, flat_1m, flat_mode):
    """Every chunk of a 1M-row scan and the hand-over ring at config 2's chunk count and batch, in
    every contraction: ids equal the oracle's for all 1,000 queries, each returned distance is the
    oracle's distance of that row, bit for bit (sampled), and no query needed the exhaustive redo."""
    base, q, ref_i = flat_1m
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    assert dev.flat_contraction() == _contraction_of(flat_mode, 128)
    assert np.array_equal(ids, ref_i)
    lib = orc.lib()
    for a in (0, 77, 255, 511, 999):
        qa = np.ascontiguousarray(q[a])
        ref_d = np.array([lib.orc_l2_f32(orc._ptr(qa), orc._ptr(base[i]), 128) for i in ids[a]], np.float32)
        assert np.array_equal(dists[a].view(np.uint32), ref_d.view(np.uint32))
    assert redo == 0


def test_calc_gt_device_matches_calc_gt(native):
    """The public device helper (the flat path behind alayalite_amd.calc_gt_device) agrees with the
    reference's float64 calc_gt (python/src/alayalite/utils.py:99-105) on continuous data."""
    import alayalite_amd
    from alayalite_amd.utils import calc_gt

    rng = np.random.default_rng(31)
    base = rng.random((4000, 300), dtype=np.float32)
    q = rng.random((25, 300), dtype=np.float32)
    ids, dists = alayalite_amd.utils.calc_gt_device(base, q, 10)
    assert ids.dtype == np.int32 and dists.shape == (25, 10)
    assert np.array_equal(ids, calc_gt(base, q, 10))


def _clib():
    import ctypes
    import os

    import alayalite_amd  # noqa: F401  (builds nothing: the in-tree library must exist)

    lib = ctypes.CDLL(os.path.join(os.path.dirname(alayalite_amd.__file__), "libalaya_hip.so"))
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.alaya_index_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.alaya_index_destroy.argtypes = [vp]
    lib.alaya_index_set_base.argtypes = [vp, vp, u64, u32, i32, vp]
    lib.alaya_index_flat_search.argtypes = [vp, vp, u64, u32, vp, vp, vp]
    lib.alaya_index_reserve.argtypes = [vp, u64]
    lib.alaya_index_write_rows.argtypes = [vp, u64, vp, u64]
    lib.alaya_index_set_valid.argtypes = [vp, u64, i32]
    lib.alaya_last_error.restype = ctypes.c_char_p
    return lib


def test_flat_tile_records_follow_updates(orc, flat_mode):
    """The single-role scan's tile records are cached on the index (f16 rows, norms, +inf for
    cleared rows): a removal (alaya_index_set_valid), a re-validation and rows written past the old
    end (alaya_index_reserve + write_rows, a partial last tile) must all reach the next flat search,
    whose answer equals the oracle's over the valid rows, in every mode."""
    import ctypes

    lib = _clib()
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rng = np.random.default_rng(808)
    n, d, k = 3000, 64, 10
    base = np.ascontiguousarray(rng.random((n, d), dtype=np.float32))
    extra = np.ascontiguousarray(rng.random((45, d), dtype=np.float32))
    q = np.ascontiguousarray(rng.random((40, d), dtype=np.float32))
    ix = ctypes.c_void_p()
    assert lib.alaya_index_create(0, ctypes.byref(ix)) == 0
    try:
        assert lib.alaya_index_set_base(ix, ptr(base), n, d, 0, None) == 0, lib.alaya_last_error()

        def flat(rows, valid):
            ids = np.zeros((len(q), k), np.uint32)
            dists = np.zeros((len(q), k), np.float32)
            redo = ctypes.c_uint32()
            assert lib.alaya_index_flat_search(ix, ptr(q), len(q), k, ptr(ids), ptr(dists),
                                               ctypes.byref(redo)) == 0, lib.alaya_last_error()
            live = np.nonzero(valid)[0]
            ref_i, ref_d = _exact(orc, rows[live], q, k)
            assert np.array_equal(ids, live[ref_i].astype(np.uint32))
            assert np.array_equal(dists.view(np.uint32), ref_d.view(np.uint32))

        valid = np.ones(n, bool)
        flat(base, valid)
        # capacity for the appended rows; this also materialises the validity bitmap
        assert lib.alaya_index_reserve(ix, n + len(extra)) == 0, lib.alaya_last_error()
        flat(base, valid)
        # remove every query's current nearest row, then put one back
        for a in range(len(q)):
            near = int(np.argmin(((base - q[a]) ** 2).sum(1)))
            assert lib.alaya_index_set_valid(ix, near, 0) == 0, lib.alaya_last_error()
            valid[near] = False
        flat(base, valid)
        back = int(np.nonzero(~valid)[0][0])
        assert lib.alaya_index_set_valid(ix, back, 1) == 0
        valid[back] = True
        flat(base, valid)
        # 45 rows appended: the last tile record is partial (3045 rows)
        assert lib.alaya_index_write_rows(ix, n, ptr(extra), len(extra)) == 0, lib.alaya_last_error()
        assert lib.alaya_index_set_valid(ix, n + 7, 1) == 0  # written rows start invalid
        rows = np.concatenate([base, extra])
        valid = np.concatenate([valid, np.zeros(len(extra), bool)])
        valid[n + 7] = True
        flat(rows, valid)
    finally:
        lib.alaya_index_destroy(ix)


@pytest.fixture(scope="module")
def flat_many(orc):
    rng = np.random.default_rng(8448)
    base = rng.random((100_000, 128), dtype=np.float32)
    q = rng.random((8448, 128), dtype=np.float32)
    ref_i, _ = orc.exact_gt(base, q, 10, num_threads=16)
    return base, q, ref_i


def test_flat_many_query_groups(native, orc, flat_many, flat_mode):
    """More query groups than the chip has block slots at 8 chunks (8,448 queries = 33 groups of
    256 in the single-role scan): the chunk count is chosen to fill whole rounds of the CUs and the
    last group is partial; the prescan runs in the -prescan modes only (3,125 records is below its
    default size).  The oracle's find_exact_gt orders equal distances by std::sort, the device by
    id, so a row whose ids differ must hold the same distances, bit for bit (ties); every returned
    distance is the oracle's distance of that row."""
    base, q, ref_i = flat_many
    dev = native.DeviceIndex(0)
    dev.set_base(base, 0)
    ids, dists, redo = dev.flat_search(q, 10)
    assert redo == 0
    lib = orc.lib()

    def d_of(a, row_ids):
        qa = np.ascontiguousarray(q[a])
        return np.array([lib.orc_l2_f32(orc._ptr(qa), orc._ptr(base[i]), 128) for i in row_ids], np.float32)

    diff = np.nonzero((ids != ref_i.astype(np.uint32)).any(1))[0]
    assert len(diff) <= len(q) // 100, len(diff)  # ties only
    for a in diff:
        got, ref = d_of(a, ids[a]), d_of(a, ref_i[a])
        assert np.array_equal(got.view(np.uint32), dists[a].view(np.uint32)), a
        assert np.array_equal(np.sort(got).view(np.uint32), np.sort(ref).view(np.uint32)), (a, ids[a], ref_i[a])
    for a in range(0, len(q), 997):
        assert np.array_equal(d_of(a, ids[a]).view(np.uint32), dists[a].view(np.uint32)), a
