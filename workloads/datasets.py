"""Seeded synthetic workloads (BASELINE.json configs; generators and seeds in SURVEY.md §8d).

GIST-shaped (C4): 1024 cluster centres ~ U[0, 0.5]^960, each point = centre + a low-rank
component (32 shared latent directions) + small isotropic noise, clipped to [0, 1].  Real GIST has
a low intrinsic dimension; purely isotropic 960-d noise would make recall 0.95 unreachable at any
practical ef, so the low-rank part is what puts recall 0.95 inside the ef sweep.
SIFT-shaped (C3): 1024 centres ~ U[0, 128)^128, point = round(centre + N(0, 12^2)) clipped [0, 255].
Text-embedding-shaped (C5): 4096 centres on the unit sphere, point = centre + low-rank component
(12 latent directions, sigma 0.15) + isotropic noise (sigma 0.002), row-normalised (inner product =
cosine).  Tuned at config 5's 10M rows (tools/sq8_recall.py, profiles/r01/c5_tuning.log): with 48
latent directions and noise 0.01 recall saturates near 0.72 at 10M (0.86 at 1M); with these values
the reference's SQ8 + rerank reaches 0.954 at ef 400.
"""

from __future__ import annotations

import numpy as np


def _chunks(n, step=65536):
    for s in range(0, n, step):
        yield s, min(n, s + step)


def gist_like(n: int, nq: int, dim: int = 960, seed_base: int = 5, seed_query: int = 6,
              n_centres: int = 1024, latent: int = 32, sigma_latent: float = 0.08,
              sigma_noise: float = 0.01):
    rng = np.random.default_rng(1234)
    centres = rng.uniform(0.0, 0.5, (n_centres, dim)).astype(np.float32)
    basis = (rng.standard_normal((latent, dim)) / np.sqrt(latent)).astype(np.float32)

    def draw(count, seed):
        r = np.random.default_rng(seed)
        out = np.empty((count, dim), np.float32)
        for s, e in _chunks(count):
            k = r.integers(0, n_centres, e - s)
            z = r.standard_normal((e - s, latent), dtype=np.float32) * sigma_latent * np.sqrt(latent)
            x = centres[k] + z @ basis
            x += r.standard_normal((e - s, dim), dtype=np.float32) * sigma_noise
            np.clip(x, 0.0, 1.0, out=out[s:e])
        return out

    return draw(n, seed_base), draw(nq, seed_query)


def sift_like(n: int, nq: int, dim: int = 128, seed_base: int = 3, seed_query: int = 4, n_centres: int = 1024):
    rng = np.random.default_rng(4321)
    centres = rng.uniform(0.0, 128.0, (n_centres, dim)).astype(np.float32)

    def draw(count, seed):
        r = np.random.default_rng(seed)
        out = np.empty((count, dim), np.float32)
        for s, e in _chunks(count):
            k = r.integers(0, n_centres, e - s)
            x = np.rint(centres[k] + r.normal(0.0, 12.0, (e - s, dim)).astype(np.float32))
            np.clip(x, 0.0, 255.0, out=out[s:e])
        return out

    return draw(n, seed_base), draw(nq, seed_query)


def text_like(n: int, nq: int, dim: int = 768, seed_base: int = 7, seed_query: int = 8,
              n_centres: int = 4096, latent: int = 12, sigma_latent: float = 0.15,
              sigma_noise: float = 0.002, centres: str = "sphere"):
    rng = np.random.default_rng(777)
    if centres == "orthant":  # GIST-style correlated centres U[0, 0.5]^dim, scaled to unit norm
        centres = rng.uniform(0.0, 0.5, (n_centres, dim)).astype(np.float32)
    elif centres == "subspace":  # topics on a 32-d subspace: neighbouring topics exist at any scale
        g = (rng.standard_normal((32, dim)) / np.sqrt(dim)).astype(np.float32)
        centres = rng.standard_normal((n_centres, 32)).astype(np.float32) @ g
    else:
        centres = rng.standard_normal((n_centres, dim)).astype(np.float32)
    centres /= np.linalg.norm(centres, axis=1, keepdims=True)
    basis = (rng.standard_normal((latent, dim)) / np.sqrt(dim)).astype(np.float32)

    def draw(count, seed):
        r = np.random.default_rng(seed)
        out = np.empty((count, dim), np.float32)
        for s, e in _chunks(count):
            k = r.integers(0, n_centres, e - s)
            z = r.standard_normal((e - s, latent), dtype=np.float32) * sigma_latent
            x = centres[k] + z @ basis
            x += r.standard_normal((e - s, dim), dtype=np.float32) * sigma_noise
            x /= np.linalg.norm(x, axis=1, keepdims=True)
            out[s:e] = x
        return out

    return draw(n, seed_base), draw(nq, seed_query)


def uniform(n: int, nq: int, dim: int, seed_base: int, seed_query: int):
    return (np.random.default_rng(seed_base).random((n, dim), dtype=np.float32),
            np.random.default_rng(seed_query).random((nq, dim), dtype=np.float32))
