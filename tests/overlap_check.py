"""Float64 restatement of the sparse poly/RBF per-pair work (PLSSVM_MI_PART_OVERLAP) on sampled rows.

For a sparse data set the K·p of a pairwise kernel splits exactly into a separable part and the
overlapping pairs (rows sharing at least one feature):

    sum_{j<m} k_ij p_j = [separable + diagonal] + O_i,   O_i = sum_{j != i, s_ij structurally != 0} c_ij p_j
    rbf : c_ij = k_ij - e_i e_j = e_i e_j expm1(2 g s_ij),  e_i = exp(-g |x_i|^2)
    poly: c_ij = (g s_ij + c0)^deg - c0^deg = sum_{k=1..deg} C(deg, k) c0^(deg-k) (g s_ij)^k

(s_ij = x_i . x_j; both forms are cancellation-free). O_i is exactly what the sparse kernels spend
their per-pair work on, while the separable part is O(m). In fp32 at the BASELINE sizes the overlap
terms are ~5e-7 of the row's K·p scale, so a full K·p check cannot see them; this
module checks O_i alone, relative to sum_j |c_ij p_j|.

Reference semantics: every pair's kernel value is part of the result
(include/plssvm/backends/HIP/svm_kernel.hip.hpp:206-268, src/plssvm/backends/OpenMP/svm_kernel.cpp:21-47).

Run as a script (``python tests/overlap_check.py CONFIG POINTS DTYPE [ALGO]``) it prints one JSON line
with the max error; tests/test_gpu_overlap.py uses that to show that ablated kernels fail the check.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

TOL = {np.float64: 1e-12, np.float32: 1e-4}


def overlap_reference(rowptr, col, val, n, d, rows, kernel, gamma, p, coef0=0.0, degree=3):
    """(O_i, sum_j |c_ij p_j|) in float64 for the sampled rows (all j < m = n - 1)."""
    m = n - 1
    Xs = sp.csr_matrix((val.astype(np.float64), col, rowptr), shape=(n, d))
    nrm = np.asarray(Xs.multiply(Xs).sum(axis=1)).ravel()
    e = np.exp(-gamma * nrm)
    XmT = Xs[:m].T.tocsc()
    p = p.astype(np.float64)
    want, scale = np.zeros(len(rows)), np.zeros(len(rows))
    for a in range(0, len(rows), 32):
        blk = rows[a:a + 32]
        G = (Xs[blk] @ XmT).tocoo()  # structure = the overlapping pairs (incl. j == i), data = s_ij
        r, j, s = G.row, G.col, G.data
        keep = j != blk[r]
        r, j, s = r[keep], j[keep], s[keep]
        if kernel == "rbf":
            c = e[blk[r]] * e[j] * np.expm1(2.0 * gamma * s)
        else:
            c = np.zeros_like(s)
            gs = gamma * s
            for k in range(1, degree + 1):
                c += math.comb(degree, k) * coef0 ** (degree - k) * gs ** k
        t = c * p[j]
        want[a:a + 32] = np.bincount(r, weights=t, minlength=len(blk))
        scale[a:a + 32] = np.bincount(r, weights=np.abs(t), minlength=len(blk))
    return want, scale


def remainder_reference(rowptr, col, val, n, d, rows, kernel, gamma, p, coef0=0.0, degree=3):
    """(R_i, sum_j |t_ij|) in float64 for the sampled rows: the kernel expansion's stored remainder alone,

        R_i = sum_{j < m, j != i, |F_i & F_j| >= 2} t_ij,   t_ij = a_i a_j H_ij p_j,
        H_ij = phi(s_ij) - sum_{f in F_i & F_j} phi(x_if x_jf)

    (F_i = the features of row i; rbf: phi(u) = expm1(2 g u), a = e; poly: phi = c, a = 1). rbf H is formed
    without cancellation from E_f = phi(x_if x_jf): 1 + E(s) = prod_f (1 + E_f), so over the shared features in
    ascending order H += P E_f, P += E_f + P E_f (P = prod - 1); poly as c(s) - sum_f c(a_f) (binomial form).
    Reference: every pair's kernel value is part of the result (svm_kernel.hip.hpp:206-268), and the expansion's
    moment terms cover exactly the single-feature parts phi(x_if x_jf)."""
    m = n - 1
    Xs = sp.csr_matrix((val.astype(np.float64), col, rowptr), shape=(n, d))
    nrm = np.asarray(Xs.multiply(Xs).sum(axis=1)).ravel()
    e = np.exp(-gamma * nrm) if kernel == "rbf" else np.ones(n)
    F = Xs[:m].T.tocsr()  # feature-major: row f = (j, x_jf), j ascending
    p = p.astype(np.float64)

    def cpoly(u):
        c = np.zeros_like(u)
        gu = gamma * u
        for k in range(1, degree + 1):
            c += math.comb(degree, k) * coef0 ** (degree - k) * gu ** k
        return c

    want, scale = np.zeros(len(rows)), np.zeros(len(rows))
    for t, i in enumerate(rows):
        fs = col[rowptr[i]:rowptr[i + 1]]
        xi = val[rowptr[i]:rowptr[i + 1]].astype(np.float64)
        sub = F[fs].tocoo()  # row k = feature fs[k] (ascending), entries (j, x_jf)
        k, j, xj = sub.row, sub.col, sub.data
        keep = j != i
        k, j, xj = k[keep], j[keep], xj[keep]
        o = np.argsort(j, kind="stable")  # per partner: its shared features in ascending order
        k, j, a = k[o], j[o], xi[k[o]] * xj[o]
        uj, st, cnt = np.unique(j, return_index=True, return_counts=True)
        sel2 = cnt >= 2
        uj, st, cnt = uj[sel2], st[sel2], cnt[sel2]
        if uj.size == 0:
            continue
        if kernel == "rbf":
            E = np.expm1(2.0 * gamma * a)
            H, P = np.zeros(uj.size), np.zeros(uj.size)
            for q in range(int(cnt.max())):
                v = q < cnt
                Eq = E[st[v] + q]
                H[v] += P[v] * Eq
                P[v] += Eq + P[v] * Eq
        else:
            s = np.array([a[b:b + c].sum() for b, c in zip(st, cnt)])
            cs = np.array([cpoly(a[b:b + c]).sum() for b, c in zip(st, cnt)])
            H = cpoly(s) - cs
        tt = e[i] * e[uj] * H * p[uj]
        want[t], scale[t] = tt.sum(), np.abs(tt).sum()
    return want, scale


# the remainder's tolerance relative to sum_j |t_ij|: bfloat16 H and bfloat16 w (expand.hip "H storage": each stored
# product moves by <= (1 + 2^-9)^2 - 1 < 2^-8 of its term; the bar leaves a factor 2), float H (float context, real-typed
# stream: H to float's relative accuracy, fp32 sums of a few hundred terms), fp64
TOL_REM = {"bf16": 2.0 ** -7, np.float32: 2e-5, np.float64: 1e-11}


def check(config, points=None, dtype=None, kernel=None, rows=256, seed=11, part="overlap", **csvm_kw):
    """One overlap (or remainder, part='remainder') K·p of the HIP path on bench.py's data for `config`,
    against the float64 restatement on `rows` sampled rows. Returns (max relative error, tolerance, info)."""
    import bench
    import plssvm_sparse_fp22_amd as pm

    cfg = bench.CONFIGS[config]
    if kernel:
        cfg = (kernel,) + tuple(cfg[1:])
    if dtype is not None:
        cfg = cfg[:3] + (dtype,) + tuple(cfg[4:])
    kern, dt = cfg[0], cfg[3]
    prm, n, d, _, extra = bench.make_problem(cfg, points, None, 0)
    if prm.val_fmt == pm._abi.VAL_FP22 and dt == np.float64:
        # FP22 storage is a float-context format: an fp64 run takes the FP22-rounded values as doubles
        from plssvm_sparse_fp22_amd import fp22

        rowptr, col, words, _, _ = prm.csr
        prm.csr = (rowptr, col, fp22.unpack(words, col.size).astype(np.float64), n, d)
        prm.val_fmt = pm._abi.VAL_REAL
        extra = dict(csr=prm.csr)
    m = n - 1
    rng = np.random.default_rng(seed)
    pv = rng.uniform(1.0, 2.0, m).astype(dt)
    sel = np.sort(rng.choice(m, rows, replace=False))
    with pm.CSVM(prm, **csvm_kw) as svm:
        svm.setup_data_on_device()
        info = svm.info()
        got = svm.kp_part(pv, part)[sel].astype(np.float64)
    rowptr, col, val, _, _ = extra["csr"]
    if prm.val_fmt == pm._abi.VAL_FP22:  # the device sees the FP22-rounded values
        from plssvm_sparse_fp22_amd import fp22

        val = fp22.unpack(prm.csr[2], val.size)
    ref = remainder_reference if part == "remainder" else overlap_reference
    want, scale = ref(rowptr, col, val.astype(dt), n, d, sel, kern, float(dt(1.0 / d)), pv,
                      coef0=float(prm.coef0), degree=prm.degree)
    if part == "remainder":
        tol = TOL_REM["bf16" if info["exp_hbytes"] == 2 else dt]
        has = scale > 0  # rows without a partner sharing two features: the device must return exactly 0
        assert has.sum() >= rows // 2, "most sampled rows must have stored remainder pairs"
        assert np.all(got[~has] == 0.0), "a row without stored pairs has a non-zero remainder"
        err = np.abs(got[has] - want[has]) / scale[has]
        return float(err.max()), tol, info
    assert scale.min() > 0, "every sampled row must have overlapping pairs"
    err = np.abs(got - want) / scale
    return float(err.max()), TOL[dt], info


if __name__ == "__main__":
    cfg, pts, dts = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    algo = sys.argv[4] if len(sys.argv) > 4 else "auto"
    part = sys.argv[5] if len(sys.argv) > 5 else "overlap"
    err, tol, info = check(cfg, pts or None, {"f32": np.float32, "f64": np.float64}[dts], sparse_algo=algo, part=part)
    print(json.dumps({"err": err, "tol": tol, "pairs": info["pairs"], "sparse_algo": info["sparse_algo"],
                      "exp_layout": info["exp_layout"], "exp_hbytes": info["exp_hbytes"]}), flush=True)
