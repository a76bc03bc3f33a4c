"""The CPU restatement (oracle/) pinned against the reference's own known answers.

Reference tests restated here:
  tests/space/raw_space_test.cpp:83-101  L2({1,2,3},{4,5,6}) == 27
  tests/space/raw_space_test.cpp:103-122 uint8 L2({183,0,0},{107,2,3}) == 5789
  tests/space/sq8_space_test.cpp:76-81   SQ8 L2 of {1,2,3,4},{5,6,7,8} == 64
  tests/simd/l2_sqr_test.cpp:292-305     SQ8 extremes, 64 dims -> 256
  tests/simd/l2_sqr_test.cpp:46-133 / ip_test.cpp  SIMD vs generic tolerance, tail dims 1..129
  tests/utils/query_utils_test.cpp:32-103 LinearPool insert/pop sequences
"""

import numpy as np
import pytest


def test_known_answer_l2(orc):
    x = np.array([1, 2, 3], np.float32)
    y = np.array([4, 5, 6], np.float32)
    assert orc.l2(x, y) == np.float32(27.0)
    assert orc.lib().orc_l2_f32_avx2(orc._ptr(x), orc._ptr(y), 3) == 27.0


def test_known_answer_uint8(orc):
    x = np.array([183, 0, 0], np.uint8)
    y = np.array([107, 2, 3], np.uint8)
    assert orc.lib().orc_l2_generic(orc._ptr(x), orc._ptr(y), 3, 2) == 5789.0


def test_known_answer_sq8(orc):
    data = np.array([[1, 2, 3, 4], [5, 6, 7, 8]], np.float32)
    mn, mx = orc.sq8_fit(data)
    codes = orc.sq8_encode(data, mn, mx)
    for variant in (0, 1, 2):
        assert orc.sq8_dist(orc.L2, codes[0], codes[1], mn, mx, variant) == pytest.approx(64.0, rel=1e-6)


def test_sq8_extremes(orc):
    x = np.zeros(64, np.uint8)
    y = np.full(64, 255, np.uint8)
    mn = np.full(64, -1.0, np.float32)
    mx = np.full(64, 1.0, np.float32)
    for variant in (0, 1, 2):
        assert orc.sq8_dist(orc.L2, x, y, mn, mx, variant) == pytest.approx(256.0, abs=1e-3)


@pytest.mark.parametrize("dim", [1, 3, 7, 8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 768, 960])
def test_avx2_order_portable_equals_intrinsics(orc, dim):
    """The portable restatement and the intrinsic restatement agree bit for bit (all tail shapes)."""
    rng = np.random.default_rng(dim)
    for _ in range(20):
        x = rng.uniform(-1, 1, dim).astype(np.float32)
        y = rng.uniform(-1, 1, dim).astype(np.float32)
        lib = orc.lib()
        a = np.float32(lib.orc_l2_f32(orc._ptr(x), orc._ptr(y), dim))
        b = np.float32(lib.orc_l2_f32_avx2(orc._ptr(x), orc._ptr(y), dim))
        assert a.view(np.uint32) == b.view(np.uint32)
        a = np.float32(lib.orc_ip_f32(orc._ptr(x), orc._ptr(y), dim))
        b = np.float32(lib.orc_ip_f32_avx2(orc._ptr(x), orc._ptr(y), dim))
        assert a.view(np.uint32) == b.view(np.uint32)


@pytest.mark.parametrize("dim", [1, 3, 17, 33, 129, 960])
def test_simd_close_to_generic(orc, dim):
    """l2_sqr_test.cpp:46-133: SIMD result within tolerance of the generic scalar loop."""
    rng = np.random.default_rng(7)
    x = rng.uniform(-1, 1, dim).astype(np.float32)
    y = rng.uniform(-1, 1, dim).astype(np.float32)
    ref = float(((x.astype(np.float64) - y) ** 2).sum())
    assert float(orc.l2(x, y)) == pytest.approx(ref, rel=1e-5, abs=1e-5)
    assert float(orc.ip(x, y)) == pytest.approx(-float((x.astype(np.float64) * y).sum()), rel=1e-4, abs=1e-4)


def _pool():
    return __import__("oracle").Pool(10, 5)


def test_pool_insert_boundary(orc):
    p = orc.Pool(10, 5)
    for i, d in [(1, 2.5), (2, 1.5), (3, 3.0), (4, 4.0), (5, 5.0)]:
        p.insert(i, d)
    assert not p.insert(6, 6.0)
    assert p.size() == 5


def test_pool_pop(orc):
    p = orc.Pool(10, 5)
    for i, d in [(1, 2.5), (2, 1.5), (3, 3.0)]:
        p.insert(i, d)
    assert p.top() == 2
    assert [p.pop(), p.pop(), p.pop()] == [2, 1, 3]


def test_pool_multiple_insert_and_pop(orc):
    p = orc.Pool(10, 5)
    for i, d in [(1, 2.5), (2, 1.5), (3, 3.0), (4, 0.5), (5, 4.0)]:
        p.insert(i, d)
    assert p.size() == 5
    assert p.pop() == 4
    p.insert(6, 2.0)
    assert [p.pop() for _ in range(5)] == [2, 6, 1, 3, 5]
    assert not p.has_next()


def test_pool_boundary_conditions(orc):
    p = orc.Pool(10, 5)
    for i, d in [(1, 2.5), (2, 1.5), (3, 3.0), (4, 0.5), (5, 4.0)]:
        p.insert(i, d)
    assert not p.insert(6, 5.0)
    assert p.size() == 5
    assert p.insert(7, -1.0)
    assert p.size() == 5


def test_pool_performance_shape(orc):
    p = orc.Pool(10, 5)
    for i in range(10000):
        p.insert(i, float(10000 - i))
    assert p.size() == 5


def test_pool_ties_go_after_existing(orc):
    p = orc.Pool(10, 4)
    p.insert(1, 1.0)
    p.insert(2, 1.0)
    p.insert(3, 0.5)
    p.insert(4, 1.0)
    assert [p.id(i) for i in range(4)] == [3, 1, 2, 4]
    assert not p.insert(5, 1.0)  # full and d >= last


def test_normalize(orc):
    v = np.array([3.0, 4.0], np.float32)
    n = orc.normalize(v)
    assert np.allclose(n, [0.6, 0.8])


def test_exact_gt_restatement(orc):
    """find_exact_gt (evaluate.hpp:29-62): l2_sqr to every row, sort by distance, first k ids."""
    rng = np.random.default_rng(11)
    base = rng.random((2000, 40), dtype=np.float32)
    q = rng.random((12, 40), dtype=np.float32)
    ids, sec = orc.exact_gt(base, q, 10, 3)
    assert sec >= 0
    for i in range(q.shape[0]):
        d = np.array([orc.l2(q[i], base[j]) for j in range(base.shape[0])], np.float32)
        assert set(ids[i].tolist()) == set(np.argsort(d, kind="stable")[:10].tolist())
