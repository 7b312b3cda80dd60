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


def check(config, points=None, dtype=None, kernel=None, rows=256, seed=11, **csvm_kw):
    """One overlap K·p of the HIP path on bench.py's data for `config`, against the float64
    restatement on `rows` sampled rows. Returns (max relative error, tolerance, info)."""
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
        got = svm.kp_part(pv, "overlap")[sel].astype(np.float64)
    rowptr, col, val, _, _ = extra["csr"]
    if prm.val_fmt == pm._abi.VAL_FP22:  # the device sees the FP22-rounded values
        from plssvm_sparse_fp22_amd import fp22

        val = fp22.unpack(prm.csr[2], val.size)
    want, scale = overlap_reference(rowptr, col, val.astype(dt), n, d, sel, kern, float(dt(1.0 / d)), pv,
                                    coef0=float(prm.coef0), degree=prm.degree)
    assert scale.min() > 0, "every sampled row must have overlapping pairs"
    err = np.abs(got - want) / scale
    return float(err.max()), TOL[dt], info


if __name__ == "__main__":
    cfg, pts, dts = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    algo = sys.argv[4] if len(sys.argv) > 4 else "auto"
    err, tol, info = check(cfg, pts or None, {"f32": np.float32, "f64": np.float64}[dts], sparse_algo=algo)
    print(json.dumps({"err": err, "tol": tol, "pairs": info["pairs"], "sparse_algo": info["sparse_algo"]}), flush=True)
