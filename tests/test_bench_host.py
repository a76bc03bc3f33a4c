"""Host-side logic of bench.py (CPU only): the operating-point search, recall, the chunked exact
ground truth (one GEMM over > 2^31 elements returned wrong neighbours at 10M x 768, so the base is
scanned in chunks) and the PMC-profile lookup."""

import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import bench  # noqa: E402


def test_choose_ef_brackets_then_bisects():
    seen = []

    def probe(ef):
        seen.append(ef)
        return ef >= 333

    ef = bench.choose_ef(probe)
    assert ef >= 333 and ef - 333 <= max(1, 200 // 100) + 1
    assert seen[:8] == [10, 20, 40, 60, 80, 120, 200, 400]
    assert bench.choose_ef(lambda ef: True) == 10
    assert bench.choose_ef(lambda ef: False) == 800


def test_recall_counts_set_intersections():
    ids = np.array([[1, 2, 3], [4, 5, 6]])
    gt = np.array([[3, 2, 9], [7, 8, 9]])
    assert bench.recall(ids, gt) == pytest.approx(2 / 6)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("chunk", [1234, 5000, 1_000_000])
def test_exact_gt_chunked_equals_brute_force(metric, chunk):
    rng = np.random.default_rng(metric)
    b = rng.random((5000, 24), dtype=np.float32)
    q = rng.random((300, 24), dtype=np.float32)
    got = bench.exact_gt(torch, torch.from_numpy(b), torch.from_numpy(q), b, q, metric=metric, chunk=chunk)
    ref = []
    for v in q.astype(np.float64):
        d = ((b.astype(np.float64) - v) ** 2).sum(1) if metric == 0 else -(b.astype(np.float64) @ v)
        ref.append(np.lexsort((np.arange(len(d)), d))[:10])
    assert np.array_equal(got, np.array(ref))


def test_pmc_traffic_picks_nearest_ef(tmp_path, monkeypatch):
    for r, ef in (("r01", 400), ("r02", 380)):
        d = tmp_path / "profiles" / r
        d.mkdir(parents=True)
        (d / "traffic.json").write_text(json.dumps({"config": {"n_base": 10, "n_queries": 2, "dim": 4, "k": 1,
                                                               "ef_search": ef}, "traffic_over_algorithmic": 1.0}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    path, t = bench.pmc_traffic({"n_base": 10, "n_queries": 2, "dim": 4, "k": 1, "ef_search": 387})
    assert t["config"]["ef_search"] == 380 and os.path.basename(os.path.dirname(path)) == "r02"
    assert bench.pmc_traffic({"n_base": 11, "n_queries": 2, "dim": 4, "k": 1, "ef_search": 387}) is None
