"""Seeded synthetic data sets.

* :func:`blobs` restates utility_scripts/generate_data.py:54-75 ("blobs": sklearn make_blobs with
  2 centres ~ U(-10, 10)^d, sigma = 1, equal classes, shuffled; labels*2-1; per-feature
  min-max scaling to [-1, 1]) with an explicit seed — the reference script is unseeded and
  crashes on sklearn >= 1.2 (list ``feature_range``), SURVEY.md Appendix C #9.
* :func:`sparse_csr` builds the sparse configs: exactly ``nnz_per_row`` columns per row, uniform
  without replacement (sorted), values clip(N(0.5*y*s_f, 0.5), -1, 1) with s_f = +-1 per feature,
  balanced labels.
"""
from __future__ import annotations

import numpy as np


def blobs(n, d, seed=1, dtype=np.float64, cluster_std=1.0):
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-10.0, 10.0, size=(2, d))
    n0 = n // 2 + n % 2
    X = np.empty((n, d), dtype=np.float64)
    X[:n0] = rng.normal(size=(n0, d)) * cluster_std + centers[0]
    X[n0:] = rng.normal(size=(n - n0, d)) * cluster_std + centers[1]
    y = np.concatenate([np.zeros(n0), np.ones(n - n0)])
    perm = rng.permutation(n)
    X, y = X[perm], y[perm]
    y = y * 2 - 1
    lo, hi = X.min(axis=0), X.max(axis=0)
    span = np.where(hi > lo, hi - lo, 1.0)
    X = (X - lo) / span * 2.0 - 1.0
    return np.ascontiguousarray(X.astype(dtype)), y.astype(dtype)


def sparse_csr(n, d, nnz_per_row, seed=3, dtype=np.float32):
    """Returns ((rowptr int64[n+1], col int32[nnz], val[nnz], n, d), y)."""
    rng = np.random.default_rng(seed)
    k = int(nnz_per_row)
    if k > d:
        raise ValueError("nnz_per_row > d")
    y = np.where(np.arange(n) % 2 == 0, 1.0, -1.0)
    rng.shuffle(y)
    s = np.where(rng.random(d) < 0.5, -1.0, 1.0)
    col = np.empty((n, k), dtype=np.int64)
    B = 1 << 18
    for a in range(0, n, B):
        e = min(n, a + B)
        c = rng.integers(0, d, size=(e - a, k))
        c.sort(axis=1)
        while True:
            dup = (np.diff(c, axis=1) == 0).any(axis=1) if k > 1 else np.zeros(e - a, bool)
            if not dup.any():
                break
            idx = np.nonzero(dup)[0]  # redraw rows with a repeated column until all are distinct
            cc = rng.integers(0, d, size=(idx.size, k))
            cc.sort(axis=1)
            c[idx] = cc
        col[a:e] = c
    val = np.empty((n, k), dtype=np.float32)
    for a in range(0, n, B):
        e = min(n, a + B)
        mu = 0.5 * y[a:e, None] * s[col[a:e]]
        val[a:e] = np.clip(rng.normal(mu, 0.5), -1.0, 1.0)
    rowptr = np.arange(0, (n + 1) * k, k, dtype=np.int64)
    return (rowptr, col.reshape(-1).astype(np.int32), val.reshape(-1).astype(dtype), n, d), y.astype(dtype)


def densify(csr, dtype=None):
    rowptr, col, val, n, d = csr
    X = np.zeros((n, d), dtype=dtype or val.dtype)
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    X[rows, col] = val
    return X
