"""Generate the committed golden fixtures under tests/golden/ (run from the repo root).

Inputs are seeded synthetic data (BASELINE config 1 shapes); the graph is built by the oracle's
restatement of HNSWBuilder::build_graph with one thread (oracle/oracle_build.cpp: hnswlib order,
seed 100); expected ids/distances/counters come from the oracle's search restatement.  Nothing here
runs the product (alayalite_amd), so the fixtures pin the engine's builders and its device search
to the restatement.  The reference itself cannot be built or run here; the
restatement is pinned to the reference by its own known-answer tests (tests/test_oracle.py).
"""

from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402

EFS = (10, 20, 50, 100)


def fixture(name, base, queries, metric, k=10):
    l0, levels, off, ue, ep, upper_r = oracle.build_hnsw(base, metric, 32, 100, 100)
    view = oracle.IndexView(base, l0, levels, off, ue, upper_r, ep, metric=metric)
    out = {"queries": queries, "l0": l0, "levels": levels, "upper_off": off, "upper_edges": ue,
           "ep": np.uint32(ep), "upper_R": np.uint32(upper_r), "metric": np.int32(metric),
           "base_md5": np.array(hashlib.md5(base.tobytes()).hexdigest()), "efs": np.array(EFS)}
    for ef in EFS:
        ids = np.zeros((len(queries), k), np.uint32)
        dists = np.zeros((len(queries), k), np.float32)
        cnt = np.zeros((len(queries), 4), np.uint64)
        for i, q in enumerate(queries):
            ids[i], dists[i], c = view.search(q, k, ef, with_counters=True)
            cnt[i] = c
        out[f"ids_ef{ef}"] = ids
        out[f"dists_ef{ef}"] = dists
        out[f"counters_ef{ef}"] = cnt
    path = os.path.join(ROOT, "tests", "golden", f"{name}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def c1_data():
    rng = np.random.default_rng(0)
    return rng.random((1000, 128), dtype=np.float32), rng.random((10, 128), dtype=np.float32)


def ip_data():
    rng = np.random.default_rng(11)
    return rng.standard_normal((800, 96)).astype(np.float32), rng.standard_normal((8, 96)).astype(np.float32)


def cos_data():
    rng = np.random.default_rng(12)
    base = rng.standard_normal((600, 100)).astype(np.float32)
    q = rng.standard_normal((8, 100)).astype(np.float32)
    for m in (base, q):
        for row in m:
            row[:] = oracle.normalize(row)
    return base, q


if __name__ == "__main__":
    fixture("c1_l2", *c1_data(), metric=oracle.L2)
    fixture("ip_96", *ip_data(), metric=oracle.IP)
    fixture("cos_100", *cos_data(), metric=oracle.COS)
