"""CPU checks of the float64 restatements tests/overlap_check.py compares the GPU with (no GPU needed).

On a small random CSR set the remainder restatement (the pairs sharing >= 2 features, H_ij = phi(s_ij) -
sum_f phi(x_if x_jf)) must equal a brute-force dense evaluation of the same definition, and the overlap sum must
split exactly into the remainder plus the single-feature (column-moment) terms sum_{f shared} phi(x_if x_jf)."""
import math

import numpy as np
import pytest
import scipy.sparse as sp

from overlap_check import overlap_reference, remainder_reference


def _set(n=300, d=40, k=6, seed=4):
    rng = np.random.default_rng(seed)
    rows = [np.sort(rng.choice(d, rng.integers(1, k + 1), replace=False)) for _ in range(n)]
    rowptr = np.zeros(n + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(0.2, 1.5, col.size)
    return rowptr, col, val, n, d


def _phi(kernel, u, gamma, coef0, degree):
    if kernel == "rbf":
        return np.expm1(2.0 * gamma * u)
    return sum(math.comb(degree, q) * coef0 ** (degree - q) * (gamma * u) ** q for q in range(1, degree + 1))


@pytest.mark.parametrize("kernel,coef0", [("rbf", 0.0), ("polynomial", 0.0), ("polynomial", 0.7)])
def test_remainder_reference_brute_force(kernel, coef0):
    rowptr, col, val, n, d = _set()
    gamma, degree = 0.3, 3
    m = n - 1
    X = sp.csr_matrix((val, col, rowptr), shape=(n, d)).toarray()
    p = np.random.default_rng(1).uniform(1.0, 2.0, m)
    rows = np.arange(0, m, 7)
    got, scale = remainder_reference(rowptr, col, val, n, d, rows, kernel, gamma, p, coef0=coef0, degree=degree)
    ov, _ = overlap_reference(rowptr, col, val, n, d, rows, kernel, gamma, p, coef0=coef0, degree=degree)
    e = np.exp(-gamma * (X * X).sum(1)) if kernel == "rbf" else np.ones(n)
    for t, i in enumerate(rows):
        want = wabs = single = 0.0
        for j in range(m):
            if j == i:
                continue
            sh = np.nonzero((X[i] != 0) & (X[j] != 0))[0]
            if sh.size == 0:
                continue
            a = X[i, sh] * X[j, sh]
            ph1 = _phi(kernel, a, gamma, coef0, degree).sum()
            single += e[i] * e[j] * ph1 * p[j]
            if sh.size >= 2:
                term = e[i] * e[j] * (_phi(kernel, a.sum(), gamma, coef0, degree) - ph1) * p[j]
                want += term
                wabs += abs(term)
        assert got[t] == pytest.approx(want, rel=1e-12, abs=1e-15)
        assert scale[t] == pytest.approx(wabs, rel=1e-12, abs=1e-15)
        assert ov[t] == pytest.approx(got[t] + single, rel=1e-11, abs=1e-14)
