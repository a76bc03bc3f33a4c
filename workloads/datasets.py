"""Seeded synthetic workloads (BASELINE.json configs; generators and seeds in SURVEY.md §8d).

GIST-shaped (C4): 1024 cluster centres ~ U[0, 0.5]^960, each point = centre + a low-rank
component (32 shared latent directions) + small isotropic noise, clipped to [0, 1].  Real GIST has
a low intrinsic dimension; purely isotropic 960-d noise would make recall 0.95 unreachable at any
practical ef, so the low-rank part is what puts recall 0.95 inside the ef sweep.
SIFT-shaped (C3): 1024 centres ~ U[0, 128)^128, point = round(centre + N(0, 12^2)) clipped [0, 255].
Text-embedding-shaped (C5): 4096 centres on the unit sphere, point = centre + low-rank component
(12 latent directions, sigma 0.15) + isotropic noise (sigma 0.002), row-normalised (inner product =
cosine); base rows drawn per 65,536-row chunk (seed [7, chunk], round 4) so any row range can be
generated alone.  Tuned at config 5's 10M rows (tools/sq8_recall.py, profiles/r01/c5_tuning.log): with 48
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


def _text_like_model(dim, n_centres, latent, centres):
    rng = np.random.default_rng(777)
    if centres == "orthant":  # GIST-style correlated centres U[0, 0.5]^dim, scaled to unit norm
        c = rng.uniform(0.0, 0.5, (n_centres, dim)).astype(np.float32)
    elif centres == "subspace":  # topics on a 32-d subspace: neighbouring topics exist at any scale
        g = (rng.standard_normal((32, dim)) / np.sqrt(dim)).astype(np.float32)
        c = rng.standard_normal((n_centres, 32)).astype(np.float32) @ g
    else:
        c = rng.standard_normal((n_centres, dim)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    basis = (rng.standard_normal((latent, dim)) / np.sqrt(dim)).astype(np.float32)
    return c, basis


def _text_like_draw(r, count, dim, c, basis, sigma_latent, sigma_noise, out):
    k = r.integers(0, c.shape[0], count)
    z = r.standard_normal((count, basis.shape[0]), dtype=np.float32) * sigma_latent
    x = c[k] + z @ basis
    x += r.standard_normal((count, dim), dtype=np.float32) * sigma_noise
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    out[:] = x


TEXT_CHUNK = 65536


def text_like_rows(lo: int, hi: int, dim: int = 768, seed_base: int = 7, n_centres: int = 4096, latent: int = 12,
                   sigma_latent: float = 0.15, sigma_noise: float = 0.002, centres: str = "sphere"):
    """Rows [lo, hi) of the text-like base.  Every 65,536-row chunk has its own generator
    (default_rng([seed_base, chunk])), so a rank generates only its own shard's rows (config 5 at
    10M x 768 is 30.7 GB of f32: 8 ranks holding the whole base would need 246 GB of host memory)."""
    import os
    from concurrent.futures import ThreadPoolExecutor

    c, basis = _text_like_model(dim, n_centres, latent, centres)
    out = np.empty((hi - lo, dim), np.float32)

    def one(ch):
        a, b = ch * TEXT_CHUNK, (ch + 1) * TEXT_CHUNK
        block = np.empty((TEXT_CHUNK, dim), np.float32)
        _text_like_draw(np.random.default_rng([seed_base, ch]), TEXT_CHUNK, dim, c, basis, sigma_latent, sigma_noise,
                        block)
        s, e = max(a, lo), min(b, hi)
        out[s - lo:e - lo] = block[s - a:e - a]

    chunks = range(lo // TEXT_CHUNK, (hi + TEXT_CHUNK - 1) // TEXT_CHUNK)
    with ThreadPoolExecutor(max(1, min(16, os.cpu_count() or 1))) as pool:  # chunks are independent
        list(pool.map(one, chunks))
    return out


def text_like_queries(nq: int, dim: int = 768, seed_query: int = 8, n_centres: int = 4096, latent: int = 12,
                      sigma_latent: float = 0.15, sigma_noise: float = 0.002, centres: str = "sphere"):
    c, basis = _text_like_model(dim, n_centres, latent, centres)
    r = np.random.default_rng(seed_query)
    out = np.empty((nq, dim), np.float32)
    for s, e in _chunks(nq):
        _text_like_draw(r, e - s, dim, c, basis, sigma_latent, sigma_noise, out[s:e])
    return out


def text_like(n: int, nq: int, dim: int = 768, seed_base: int = 7, seed_query: int = 8,
              n_centres: int = 4096, latent: int = 12, sigma_latent: float = 0.15,
              sigma_noise: float = 0.002, centres: str = "sphere"):
    kw = dict(n_centres=n_centres, latent=latent, sigma_latent=sigma_latent, sigma_noise=sigma_noise, centres=centres)
    return (text_like_rows(0, n, dim, seed_base, **kw), text_like_queries(nq, dim, seed_query, **kw))


def uniform(n: int, nq: int, dim: int, seed_base: int, seed_query: int):
    return (np.random.default_rng(seed_base).random((n, dim), dtype=np.float32),
            np.random.default_rng(seed_query).random((nq, dim), dtype=np.float32))
